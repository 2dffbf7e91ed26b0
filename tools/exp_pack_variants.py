"""Experiment builds of pw_pack.hip (never shipped), linked with the other product objects into
tools/abl_build/<name>/lib for tools/pk_sweep.sh (PWASM_LIB):
  cur      the working copy
  head     pw_pack.hip as committed at git HEAD (the A of an A/B against an uncommitted edit)
  pkg<N>   pack_cs_kernel grid capped at N workgroups per CU (product: 64)
  stream / s5 / s6 / s7  the stream packer (profiles/variants/pack_stream_tasks.patch), held to 5-7 waves/SIMD
  k<N>     N records per task (stream patch builds; 8)
  w8       the kernel held to 8 waves/SIMD (amdgpu_waves_per_eu: SGPRs spilled to VGPR lanes)
Usage: python tools/exp_pack_variants.py [names...]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "pwasm_amd/csrc/pw_pack.hip")
OUT = os.path.join(REPO, "tools/abl_build")
TMP = os.path.join(REPO, "build_exp")


def make(name):
    s = open(SRC).read()
    if name == "head":
        s = subprocess.run(["git", "-C", REPO, "show", "HEAD:pwasm_amd/csrc/pw_pack.hip"], capture_output=True, text=True,
                           check=True).stdout
    elif name.startswith("pkg"):
        old = "const uint32_t cap = (uint32_t)ncu * 64u;"
        assert old in s
        s = s.replace(old, f"const uint32_t cap = (uint32_t)ncu * {int(name[3:])}u;")
    elif name == "w8":  # amdgpu_waves_per_eu(8): SGPRs <= 96 (more spilled to VGPR lanes), 8 waves/SIMD
        old = "__global__ __launch_bounds__(256) void pack_cs_kernel"
        assert old in s
        s = s.replace(old, "__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void pack_cs_kernel")
    elif name in ("stream", "s5", "s6", "s7"):  # profiles/variants/pack_stream_tasks.patch (+ waves/SIMD held)
        os.makedirs(TMP, exist_ok=True)
        p = os.path.join(TMP, f"pack_{name}_base.hip")
        open(p, "w").write(s)
        subprocess.run(["patch", "-s", p, os.path.join(REPO, "profiles/variants/pack_stream_tasks.patch")], check=True)
        s = open(p).read()
        if name != "stream":
            old = "__global__ __launch_bounds__(256) void pack_cs_kernel"
            assert old in s
            s = s.replace(old, f"__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu({name[1]}, {name[1]}))) void pack_cs_kernel")
    elif name == "pk_nt":  # cs text loads non-temporal
        for k in ("  d0 = *reinterpret_cast<const uint32_t*>(text + (a0 < last ? a0 : last));",
                  "  d1 = *reinterpret_cast<const uint32_t*>(text + (a0 + 4 < last ? a0 + 4 : last));"):
            assert k in s
            s = s.replace(k, k.replace("*reinterpret_cast<const uint32_t*>(", "__builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(").replace(";", ");", 1) if False else
                          k.replace("= *reinterpret_cast<const uint32_t*>(text + ", "= __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(text + ").replace("));", ")));"))
    elif name.startswith("k") and name[1:].isdigit():  # records per task (product: 8)
        old = "constexpr uint32_t kTaskRecs = 8;"
        assert old in s
        s = s.replace(old, f"constexpr uint32_t kTaskRecs = {int(name[1:])};")
    elif name != "cur":
        raise SystemExit(f"unknown variant {name}")
    os.makedirs(TMP, exist_ok=True)
    p = os.path.join(TMP, f"pack_{name}.hip")
    open(p, "w").write(s)
    return p


def build(name):
    src = make(name)
    bdir = os.path.join(REPO, "pwasm_amd/build")
    objs = [os.path.join(bdir, f) for f in sorted(os.listdir(bdir)) if f.endswith(".o") and f != "pw_pack.o"]
    inc = ["-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "pwasm_amd/csrc")]
    d = os.path.join(OUT, name)
    os.makedirs(os.path.join(d, "lib"), exist_ok=True)
    o = os.path.join(d, "pw_pack.o")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall",
                    "-Wno-unused-function", *inc, "-c", src, "-o", o], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                    os.path.join(d, "lib", "libpwasm_amd.so"), o, *objs, "-ldl"], check=True)
    print("built", name, flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or ["cur"]:
        build(n)
