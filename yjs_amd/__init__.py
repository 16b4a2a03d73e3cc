"""yjs_amd -- MI355X-native batched Yjs update engine.

Python host mirror of the yjs binary update API (yjs 13.5.16 names, gaberogan/yjs@v0 wire format),
backed by libymerge.so (HIP kernels for gfx950).  There is no CPU fallback: every call runs on the
GPU and fails loudly when the extension or the device is missing.
"""
from .engine import (  # noqa: F401
    Engine, YjsError, YjsURIError, YjsTypeError, YjsRangeError, YjsSyntaxError, UnsupportedInput,
    mergeUpdates, mergeUpdatesV2, diffUpdate, diffUpdateV2,
    encodeStateVectorFromUpdate, encodeStateVectorFromUpdateV2,
    mergeUpdatesBatch, diffUpdateBatch, encodeStateVectorFromUpdateBatch,
    convertUpdateFormatV1ToV2, convertUpdateFormatV2ToV1, convertUpdateFormatBatch,
    parseUpdateMeta, parseUpdateMetaV2, parseUpdateMetaBatch, decode_meta,
    mergeDeleteSetsBatch, mergeEncodedDeleteSets,
    Snapshot, convertSnapshotBatch, decodeSnapshotBatch, encodeSnapshotBatch,
    decodeSnapshot, decodeSnapshotV2, encodeSnapshot, encodeSnapshotV2,
    compactUpdates, compactUpdatesV2, compactUpdatesBatch,
    pack_docs, lib_path, status_class, status_message,
)
