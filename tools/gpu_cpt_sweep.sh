#!/bin/bash
# compaction launch-shape sweep: YMERGE_COMPACT_LANES x YMERGE_COMPACT_OCC over the compaction bench lines
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for occ in ${OCCS:-1 2}; do
  YMERGE_COMPACT_OCC=$occ TAG=${TAG:-cpt}_o$occ VAR=YMERGE_COMPACT_LANES VALS="${LANES:-4 8 16 32}" SEC=${SEC:-compact_c2_v1,compact_c4_v1} bash tools/env_sweep.sh | sed "s/^/occ=$occ /"
done
