"""Source hash of libsepvad.so: sha256 over the C ABI header and every file the library is compiled from.

The Makefile runs this script to write ``csrc/build/build_id.h`` (the value ``sepvad_build_id()`` returns), and the
tests recompute it from the tree, so a library built from other sources than the tree it is tested in is caught
(VERDICT r05 item 5). Files are hashed in sorted relative-path order as ``path NUL content NUL``.

usage: python buildid.py            -> prints the hash
       python buildid.py --header F -> writes F (``#define SEPVAD_BUILD_ID "<hash>"``) if its content changed
"""
from __future__ import annotations

import hashlib
import os
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)


def source_files(repo: str = REPO) -> list[str]:
    """Repository-relative paths of the library's sources: csrc/*.hip, csrc/*.h, csrc/Makefile, include/sepvad.h."""
    csrc = os.path.join(repo, "sep-tfanet-vad_amd", "csrc")
    rel = [os.path.join("sep-tfanet-vad_amd", "csrc", f) for f in os.listdir(csrc)
           if f.endswith((".hip", ".h")) or f == "Makefile"]
    rel.append(os.path.join("include", "sepvad.h"))
    return sorted(p.replace(os.sep, "/") for p in rel)


def source_hash(repo: str = REPO) -> str:
    h = hashlib.sha256()
    for rel in source_files(repo):
        with open(os.path.join(repo, rel), "rb") as f:
            data = f.read()
        h.update(rel.encode() + b"\0" + data + b"\0")
    return h.hexdigest()[:16]


def main(argv: list[str]) -> None:
    hid = source_hash()
    if "--header" in argv:
        path = argv[argv.index("--header") + 1]
        text = f'#pragma once\n#define SEPVAD_BUILD_ID "{hid}"\n'
        old = open(path).read() if os.path.exists(path) else None
        if old != text:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            with open(path, "w") as f:
                f.write(text)
    else:
        print(hid)


if __name__ == "__main__":
    main(sys.argv[1:])
