"""Golden vectors for the Boost text-archive writer: the SHA-256 and byte size
of every tree file the reference ships (data/trees_headpose/tree_NNN.txt, data/trees_ffd/forest_F/
tree_NNN.txt), keyed by the path each archive records as its m_save_path.  Generated from
/root/reference's own files (read as data); tests/test_archive.py checks that
ffd_model_tree_archive re-emits exactly these bytes from the converted model.

    python tests/golden/make_archive_digests.py [/root/reference]
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = {}
    for sub in ("data/trees_headpose", "data/trees_ffd"):
        for dirpath, _, files in sorted(os.walk(os.path.join(ref, sub))):
            for f in sorted(files):
                if f.startswith("tree_") and f.endswith(".txt"):
                    p = os.path.join(dirpath, f)
                    b = open(p, "rb").read()
                    out[os.path.relpath(p, ref)] = {"sha256": hashlib.sha256(b).hexdigest(), "bytes": len(b)}
    json.dump(dict(sorted(out.items())), open(os.path.join(HERE, "archive_digests.json"), "w"), indent=1)
    print(f"{len(out)} tree files")


if __name__ == "__main__":
    main()
