"""SHA-256 of the sources libgsr.so is built from (3dgs_study_amd/csrc/*.hip,
*.hpp, Makefile and include/gsr.h, in name order, each as name + NUL + bytes).
The Makefile compiles it into the library (gsr_build_id); tests/test_abi.py
checks that the shipped library matches the tree it ships with."""
import hashlib
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def sources():
    csrc = ROOT / "3dgs_study_amd" / "csrc"
    files = sorted(list(csrc.glob("*.hip")) + list(csrc.glob("*.hpp")) + [csrc / "Makefile"])
    return files + [ROOT / "include" / "gsr.h"]


def build_id() -> str:
    h = hashlib.sha256()
    for f in sources():
        h.update(f.relative_to(ROOT).as_posix().encode() + b"\0")
        h.update(f.read_bytes())
    return h.hexdigest()


if __name__ == "__main__":
    sys.stdout.write(build_id())
