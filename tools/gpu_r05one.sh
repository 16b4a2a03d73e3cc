set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
export YMERGE_DF2_ONE=1
for w in c2r_v2 c4r_v2; do OP=diff WL=$w timeout -k 10 120 python3 tools/pv2_reasons.py 2>&1 | tail -1; done
TAG=r05one WLS="c2r_v2 c4r_v2" OP=diff NDOCS=4096 TOPK=6 bash tools/kstat_wl.sh 2>&1 | grep -v "^[EW]2026"
