"""Experiment builds of pw_msa.hip (never shipped): `python tools/exp_msa.py name=path.hip ...`
links each source with the other product objects into tools/abl_build/<name>/lib, for
tools/exp_sweep.sh (BENCH_ARGS="--config 5") to time under the same bench (PWASM_LIB)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tools/abl_build")


def main(args):
    bdir = os.path.join(REPO, "pwasm_amd/build")
    objs = [os.path.join(bdir, f) for f in sorted(os.listdir(bdir)) if f.endswith(".o") and f != "pw_msa.o"]
    inc = ["-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "pwasm_amd/csrc")]
    for a in args:
        name, path = a.split("=", 1)
        d = os.path.join(OUT, name)
        os.makedirs(os.path.join(d, "lib"), exist_ok=True)
        o = os.path.join(d, "pw_msa.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall",
                        "-Wno-unused-function", *inc, "-c", path, "-o", o], check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                        os.path.join(d, "lib", "libpwasm_amd.so"), o, *objs, "-ldl"], check=True)
        print("built", name, flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
