"""Experiment builds (never shipped): variants of pw_report.hip — the committed HEAD version, the
working copy, splices of the two and patched copies — linked into tools/abl_build/<name>/lib so
tools/exp_sweep.sh can time each one's kernels under the same bench (PWASM_LIB)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "pwasm_amd/csrc/pw_report.hip")
OUT = os.path.join(REPO, "tools/abl_build")
TC_BEGIN = "constexpr int kTcOps"
TC_END = "// ------------------------------------------------------------------ fixup_kernel"


def head_src():
    return subprocess.run(["git", "show", "HEAD:pwasm_amd/csrc/pw_report.hip"], cwd=REPO, check=True,
                          capture_output=True, text=True).stdout


def splice(dst, src, a, b):
    """dst with its [a, b) region replaced by src's"""
    i, j = dst.index(a), dst.index(b)
    k, l = src.index(a), src.index(b)
    return dst[:i] + src[k:l] + dst[j:]


def patched(s, pairs):
    for a, b in pairs:
        assert a in s, a
        s = s.replace(a, b)
    return s


def variants():
    """name -> source text; edit this table per experiment (splice(), patched())"""
    cur, head = open(SRC).read(), head_src()
    return {
        "head": head,
        "cur": cur,
    }


def main(names):
    vs = variants()
    objs = [os.path.join(REPO, "pwasm_amd/build", f) for f in sorted(os.listdir(os.path.join(REPO, "pwasm_amd/build")))
            if f.endswith(".o") and f != "pw_report.o"]
    for name in names or list(vs):
        d = os.path.join(OUT, name)
        os.makedirs(os.path.join(d, "lib"), exist_ok=True)
        hip = os.path.join(d, "pw_report.hip")
        open(hip, "w").write(vs[name])
        o = os.path.join(d, "pw_report.o")
        inc = ["-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "pwasm_amd/csrc")]
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall",
                        "-Wno-unused-function", *inc, "-c", hip, "-o", o], check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                        os.path.join(d, "lib", "libpwasm_amd.so"), o, *objs, "-ldl"], check=True)
        print("built", name, flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
