"""A/B builds for same-box comparisons: librlmd_amd.so with some sources taken
from another git revision, linked against the current build's other objects.

    python tools/ab_build.py <rev> <tag> rows.hip [more.hip | header.h ...]
writes tools/_abh/librlmd_amd_<tag>.so; load it with RLMD_LIB_PATH=<that path>
(rlmd_amd/_abi.py), e.g. bench.py A/B runs on one box."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rlmd_amd import build as B  # noqa: E402

OUT = os.path.join(ROOT, "tools", "_abh")


def main():
    rev, tag, files = sys.argv[1], sys.argv[2], sys.argv[3:]
    B.build()
    src_dir = os.path.join(OUT, tag)
    os.makedirs(src_dir, exist_ok=True)
    # headers from the revision sit beside its sources: a quoted #include finds them first
    for h in [f for f in files if f.endswith(".h")]:
        text = subprocess.run(["git", "show", f"{rev}:rlmd_amd/csrc/{h}"], cwd=ROOT, capture_output=True, text=True,
                              check=True).stdout
        with open(os.path.join(src_dir, h), "w") as f:
            f.write(text)
    objs = []
    for src in B.SOURCES:
        if src in files:
            text = subprocess.run(["git", "show", f"{rev}:rlmd_amd/csrc/{src}"], cwd=ROOT, capture_output=True,
                                  text=True, check=True).stdout
            path = os.path.join(src_dir, src)
            with open(path, "w") as f:
                f.write(text)
            obj = os.path.join(src_dir, src.replace(".hip", ".o"))
            cmd = [B.HIPCC, *B.FLAGS, *B.PER_FILE.get(src, B.DEFAULT_EXTRA), f"-I{B.CSRC}",
                   f"-I{os.path.join(ROOT, 'include')}", "-c", path, "-o", obj]
            subprocess.run(cmd, check=True)
            objs.append(obj)
        else:
            objs.append(os.path.join(B.BUILD, src.replace(".hip", ".o")))
    lib = os.path.join(OUT, f"librlmd_amd_{tag}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib, *objs], check=True)
    print("built", lib)


if __name__ == "__main__":
    main()
