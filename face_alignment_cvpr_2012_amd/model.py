"""Read-only numpy view of an FFDMODEL container (include/ffd_model_format.h).

Used by tests and tools; the engine reads the same file natively (csrc/model_io.hpp).
"""
import numpy as np

_DT = {"i8": np.int8, "u8": np.uint8, "i16": np.int16, "i32": np.int32, "i64": np.int64, "f32": np.float32,
       "f64": np.float64}
_ENTRY = np.dtype([("name", "S48"), ("dtype", "S8"), ("ndim", "<u4"), ("pad", "<u4"), ("shape", "<u8", (4,)),
                   ("offset", "<u8"), ("nbytes", "<u8")])


def load(path):
    """Return {array name: numpy array} (memory-mapped, read-only)."""
    mm = np.memmap(path, dtype=np.uint8, mode="r")
    if bytes(mm[:8]) != b"FFDMODEL":
        raise ValueError(f"{path}: not an FFDMODEL file")
    ver, n = np.frombuffer(mm[8:16], "<u4")
    if ver != 1:
        raise ValueError(f"{path}: unsupported version {ver}")
    ents = np.frombuffer(mm[16:16 + n * _ENTRY.itemsize], _ENTRY)
    out = {}
    for e in ents:
        shape = tuple(int(v) for v in e["shape"][: e["ndim"]])
        dt = _DT[e["dtype"].decode()]
        a = np.frombuffer(mm, dtype=dt, count=int(np.prod(shape)) if shape else 1, offset=int(e["offset"]))
        out[e["name"].decode()] = a.reshape(shape)
    return out


def tree_stats(m, prefix, tree):
    """(nodes, leaves, sum of thresholds) of one tree — the known-answer values of SURVEY.md App. C."""
    off = m[prefix + ".tree_node_off"]
    b, e = int(off[tree]), int(off[tree + 1])
    leaf = m[prefix + ".node_leaf"][b:e]
    thr = m[prefix + ".node_split"][b:e, 9].astype(np.int64)
    return e - b, int((leaf >= 0).sum()), int(thr.sum())
