"""Experiment variants of pw_report.hip (never shipped; timing only unless noted) linked into
tools/abl_build/<name>/lib for tools/exp_sweep.sh (PWASM_LIB):
  cur      the working copy
  allgen   every render wave takes the general emit_event path (same bytes)
  allfast  every render wave takes emit_fast (wrong bytes where a lane is not fast: timing only)
  noline   no line is built (every line 78 bytes of whatever the buffer holds: timing only)
  nowin    the per-lane query window is not loaded (constant bytes: timing only)
  nohot    the Hot records are replaced by synthetic insertions after the load (timing only)
  nocopy   render's copy-out (LDS page image + stores) skipped (timing only)
  fx_inline  fixup_kernel reads outside its windows inline (no out-of-line call per byte)
  fx_bigwin  fixup_kernel stages 128 query bytes and 64 literal bytes per line
  tc_nowalk  tctx_kernel skips the op walk (timing only)
  ls148    148-byte line buffer stride (odd dword count: fewer LDS bank conflicts between lanes)
Usage: python tools/exp_report_variants.py [names...]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "pwasm_amd/csrc/pw_report.hip")
OUT = os.path.join(REPO, "tools/abl_build")
TMP = os.path.join(REPO, "build_exp")

PATCHES = {
    "cur": [],
    "allgen": [("      if (__ballot(!fast) == 0) {\n        DLine dl;", "      if (false) {\n        DLine dl;")],
    "allfast": [("      if (__ballot(!fast) == 0) {\n        DLine dl;", "      if (true) {\n        DLine dl;")],
    "noline": [("      if (__ballot(!fast) == 0) {\n        DLine dl;",
                "      if (A.n_alns != 0) {\n        merr = -1;\n        linelen = 78;\n      } else if (__ballot(!fast) == 0) {\n        DLine dl;")],
    "nowin": [("  for (int q = 0; q < kQWin / 16; q++) p.q[q] = a0[q];\n  p.qlo = x0a;",
               "  for (int q = 0; q < kQWin / 16; q++) p.q[q] = (v4u){0x41434741u, 0x54414341u, 0x47544341u, 0x41434741u};\n  p.qlo = x0a;")],
    "nohot": [("  r.a = p[0];\n  r.b = p[1];\n  return r;", "  r.a = p[0];\n  r.b = p[1];\n  if (cc > 60000000) return r;\n  r.a = (v4u){0u, 2000u, 100u + 64u * (uint32_t)(cc & 15u) + lane, 50u};\n  r.b = (v4u){0u, (uint32_t)(PW_OP_INS << 30) | (1u << 28) | kFnAcgt | 2u, 0x41414141u, 0x41414141u};\n  return r;")],
    "nocopy": [("      if (B + (uint32_t)kPageSlack <= (uint32_t)PW_PAGE_BYTES) {  // (uniform) the page in place:",
                "      if (A.n_alns != 0) {\n      } else if (B + (uint32_t)kPageSlack <= (uint32_t)PW_PAGE_BYTES) {")],
    # fixup_kernel: the global fallbacks of its Rec inline (RecFix), or 128-byte query / 64-byte
    # literal windows instead of 48 / 32
    "fx_inline": [("struct RecFast : Rec {\n  static constexpr bool kFast = true;\n};",
                   "struct RecFast : Rec {\n  static constexpr bool kFast = true;\n};\nstruct RecFix : Rec {};"),
                  ("__device__ __forceinline__ uint8_t Rc(const RecFast& r, int x) { return r.qw[x - r.qlo]; }",
                   "__device__ __forceinline__ uint8_t Rc(const RecFast& r, int x) { return r.qw[x - r.qlo]; }\n"
                   "__device__ __forceinline__ uint8_t Rc(const RecFix& r, int x) {\n  const unsigned o = (unsigned)(x - r.qlo);\n"
                   "  if (o < (unsigned)r.qn) return r.qw[o];\n  return (unsigned)x < (unsigned)r.L ? r.R[x] : (uint8_t)0;\n}\n"
                   "__device__ __forceinline__ uint8_t litb(const RecFix& r, uint32_t i) {\n  const uint32_t o = i - r.ls0;\n"
                   "  if (o < r.ln) return (uint8_t)((o < 4 ? r.lit0 : r.lit1) >> (8 * (o & 3)));\n  const uint32_t ow = i - r.l_lo;\n"
                   "  if (ow < r.l_n) return r.lw[ow];\n  return r.lits[i];\n}"),
                  ("    Rec r;\n    r.lits = A.lits;\n    r.R = A.qseq + ((uint64_t)h.qb << 4);\n    r.L = h.L;\n    r.NS = A.next_stop ? A.next_stop + ((uint64_t)h.qb << 4) : nullptr;\n    r.tab = tp;",
                   "    RecFix r;\n    r.lits = A.lits;\n    r.R = A.qseq + ((uint64_t)h.qb << 4);\n    r.L = h.L;\n    r.NS = A.next_stop ? A.next_stop + ((uint64_t)h.qb << 4) : nullptr;\n    r.tab = tp;")],
    # line buffers at an odd dword stride (148 bytes: lanes at the same line position hit 32 distinct
    # banks instead of 16), the copy-out then reading each line with 4-byte-aligned loads
    "ls148": [("constexpr int kLStride = 144;", "constexpr int kLStride = 148;"),
              ("        const LDS v4u* lp4 = reinterpret_cast<const LDS v4u*>(my_line);",
               "        const LDS v4a4* lp4 = reinterpret_cast<const LDS v4a4*>(my_line);")],
    # tctx_kernel without the op walk (an 11-byte record of whatever the buffer holds: timing only)
    "tc_nowalk": [("      emit_tctx_walk(ks, r, wd >> 30, ne, (uint32_t)j, wd, (int)p0.w, (int)p1.x, h.ls);",
                   "      if (A.n_alns == 0) emit_tctx_walk(ks, r, wd >> 30, ne, (uint32_t)j, wd, (int)p0.w, (int)p1.x, h.ls);\n      else ks.pos = 11;")],
    "fx_bigwin": [("constexpr int kFxLit = 32;", "constexpr int kFxLit = 64;\nconstexpr int kFxQ = 128;"),
                  ("  uint8_t qw[kQWin];\n  uint8_t lw[kFxLit];", "  uint8_t qw[kFxQ];\n  uint8_t lw[kFxLit];"),
                  ("    for (int q = 0; q < kQWin / 16; q++) *reinterpret_cast<LDS v4u*>(me->qw + 16 * q) = a0[q];",
                   "    for (int q = 0; q < kFxQ / 16; q++) *reinterpret_cast<LDS v4u*>(me->qw + 16 * q) = a0[q];"),
                  ("    r.qw = me->qw;\n    r.qlo = x0a;\n    r.qn = kQWin;", "    r.qw = me->qw;\n    r.qlo = x0a;\n    r.qn = kFxQ;")],
}


def build(name):
    s = open(SRC).read()
    for a, b in PATCHES[name]:
        assert a in s, (name, a)
        s = s.replace(a, b)
    os.makedirs(TMP, exist_ok=True)
    src = os.path.join(TMP, f"report_{name}.hip")
    open(src, "w").write(s)
    d = os.path.join(OUT, name)
    os.makedirs(os.path.join(d, "lib"), exist_ok=True)
    o = os.path.join(d, "pw_report.o")
    inc = ["-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "pwasm_amd/csrc")]
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall",
                    "-Wno-unused-function", "-mllvm", "-amdgpu-sched-strategy=max-memory-clause", *inc, "-c", src,
                    "-o", o], check=True)
    bdir = os.path.join(REPO, "pwasm_amd/build")
    objs = [os.path.join(bdir, f) for f in sorted(os.listdir(bdir)) if f.endswith(".o") and f != "pw_report.o"]
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                    os.path.join(d, "lib", "libpwasm_amd.so"), o, *objs, "-ldl"], check=True)
    print("built", name, flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(PATCHES):
        build(n)
