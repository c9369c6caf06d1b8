"""Boost text-archive writer over the C ABI.

Python mirror of the reference's `Tree<S>::save` (/root/reference/include/Tree.hpp:239-256), which
writes `boost::archive::text_oarchive << *this` to the tree's `m_save_path`.  The bytes come from
`ffd_model_tree_archive` / `ffd_model_save_tree` in libffd.so (csrc/ffd_archive.cpp); for the
converted pretrained model they equal the reference's shipped `data/trees_*/.../tree_NNN.txt` files.

    python -m face_alignment_cvpr_2012_amd.archive model/ffd_model.bin OUT_ROOT
writes every tree to OUT_ROOT/<m_save_path> (e.g. OUT_ROOT/data/trees_ffd/forest_0/tree_000.txt).
"""
import ctypes
import os
import sys

from . import FFDError, lib

HEADPOSE, FFD = 0, 1


class ModelArchive:
    """An opened FFDMODEL container whose trees can be re-emitted as Boost text archives."""

    def __init__(self, path):
        L = lib()
        h = ctypes.c_void_p()
        st = L.ffd_model_open(os.fsencode(path), ctypes.byref(h))
        if st != 0:
            raise FFDError(st, L.ffd_model_last_error().decode())
        self._h = h

    def close(self):
        if self._h:
            lib().ffd_model_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st):
        if st != 0:
            raise FFDError(st, lib().ffd_model_last_error().decode())

    def num_trees(self, kind):
        return int(lib().ffd_model_num_trees(self._h, kind))

    def save_path(self, kind, tree):
        buf = ctypes.create_string_buffer(4096)
        self._check(lib().ffd_model_tree_save_path(self._h, kind, tree, buf, len(buf)))
        return buf.value.decode()

    def tree_bytes(self, kind, tree):
        """The archive text of one tree (what Tree<S>::save writes), as bytes."""
        n = ctypes.c_int64()
        self._check(lib().ffd_model_tree_archive(self._h, kind, tree, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        self._check(lib().ffd_model_tree_archive(self._h, kind, tree, buf, n.value, ctypes.byref(n)))
        return buf.raw[: n.value]

    def save_tree(self, kind, tree, path):
        self._check(lib().ffd_model_save_tree(self._h, kind, tree, os.fsencode(path)))

    def save_all(self, out_root):
        """Every tree to out_root/<its m_save_path>; returns the written paths."""
        written = []
        for kind in (HEADPOSE, FFD):
            for t in range(self.num_trees(kind)):
                dst = os.path.join(out_root, self.save_path(kind, t))
                os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
                self.save_tree(kind, t, dst)
                written.append(dst)
        return written


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 2:
        print("usage: python -m face_alignment_cvpr_2012_amd.archive <model.bin> <out_root>", file=sys.stderr)
        return 2
    with ModelArchive(argv[0]) as m:
        paths = m.save_all(argv[1])
    print(f"wrote {len(paths)} trees under {argv[1]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
