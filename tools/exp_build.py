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


PROBE = "{ const uint64_t t_ = __builtin_amdgcn_s_memtime(); pa.t[%d] += t_ - pa.last; pa.last = t_; }"
PROF_PATCH = [
    ("struct ClampSink {\n", """struct ProfAcc {
  uint64_t t[16];
  uint64_t last;
};
__device__ unsigned long long g_prof[16];
struct ClampSink {
  ProfAcc* pa;
  __device__ __forceinline__ void probe(int i) {
    const uint64_t t_ = __builtin_amdgcn_s_memtime();
    pa->t[i] += t_ - pa->last;
    pa->last = t_;
  }
"""),
    ("typedef ClampSink LineSink;\n", """typedef ClampSink LineSink;
template <class S>
__device__ __forceinline__ void sink_probe(S&, int) {}
__device__ __forceinline__ void sink_probe(ClampSink& k, int i) { k.probe(i); }
"""),
    ("  // ---- bases field (\"[n]\" past MAX_EVLEN", "  sink_probe(k, 1);\n  // ---- bases field (\"[n]\" past MAX_EVLEN"),
    ("  // ---- \"E\\trloc\\taapos(aa)\\t\"", "  sink_probe(k, 11);\n  // ---- \"E\\trloc\\taapos(aa)\\t\""),
    ("      indel_impact(k, r, e, in.ns_pre);", "      sink_probe(k, 13);\n      indel_impact(k, r, e, in.ns_pre);"),
    ("  if (stop_i >= 0) {", "  sink_probe(k, 12);\n  if (stop_i >= 0) {"),
    ("  // ---- target context (setTContext", "  sink_probe(k, 2);\n  // ---- target context (setTContext"),
    ("  k.put('\\t');\n  // ---- query context", "  k.put('\\t');\n  sink_probe(k, 3);\n  // ---- query context"),
    ("  // ---- codon consequence (predictImpact", "  sink_probe(k, 4);\n  // ---- codon consequence (predictImpact"),
    ("  k.put('\\n');\n  return modseq_err;", "  sink_probe(k, 5);\n  k.put('\\n');\n  return modseq_err;"),
    ("  for (; c < W.n_chunks; c += nw) {\n", "  ProfAcc pa = {};\n  pa.last = __builtin_amdgcn_s_memtime();\n  for (; c < W.n_chunks; c += nw) {\n    " + (PROBE % 10) + "\n"),
    ("      LineSink k;\n", "      LineSink k;\n      k.pa = &pa;\n"),
    ("      const int merr = emit_event(k, r, in, skip, rel);", "      " + (PROBE % 0) + "\n      const int merr = emit_event(k, r, in, skip, rel);"),
    ("    render_pre(A, W, h, (c + nw) * kWave + (uint64_t)lane, skip, pre);\n",
     "    " + (PROBE % 6) + "\n    render_pre(A, W, h, (c + nw) * kWave + (uint64_t)lane, skip, pre);\n    " + (PROBE % 7) + "\n"),
    ("    if (ok && B > 0) {\n", "    " + (PROBE % 8) + "\n    if (ok && B > 0) {\n"),
    ("      for (uint32_t cc = (uint32_t)lane * 16; cc < B; cc += kWave * 16) {",
     "      " + (PROBE % 9) + "\n      for (uint32_t cc = (uint32_t)lane * 16; cc < B; cc += kWave * 16) {"),
    ("    wave_sync();\n  }\n}\n\n// ------------------------------------------------------------------ tctx_kernel",
     "    wave_sync();\n  }\n  if (lane == 0)\n    for (int i = 0; i < 16; i++) atomicAdd(&g_prof[i], (unsigned long long)pa.t[i]);\n}\n\n// ------------------------------------------------------------------ tctx_kernel"),
]
PROF_HOST = """
extern "C" int pw_exp_prof(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pw::g_prof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  unsigned long long z[16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(pw::g_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
"""


# counts of render waves on the fast / general emit_event instantiation and their lanes
# (tools/exp_fastcnt.py): g_prof[0] fast waves, [1] general waves, [2] lanes not fast, [3] active
FASTCNT_PATCH = [
    ("struct ClampSink {\n", "__device__ unsigned long long g_prof[16];\nstruct ClampSink {\n"),
    ("      if (__ballot(!fast) == 0) {",
     "      {\n        const uint64_t bf_ = __ballot(!fast), ba_ = __ballot(true);\n"
     "        if ((uint32_t)lane == (uint32_t)__builtin_ctzll(ba_)) {\n"
     "          atomicAdd(&g_prof[bf_ == 0 ? 0 : 1], 1ull);\n"
     "          atomicAdd(&g_prof[2], (unsigned long long)__popcll(bf_));\n"
     "          atomicAdd(&g_prof[3], (unsigned long long)__popcll(ba_));\n        }\n      }\n"
     "      if (__ballot(!fast) == 0) {"),
]
TG = "    if (tg > (uint64_t)ncu * 4u) tg = (uint64_t)ncu * 4u;"


def profiled(s):
    return patched(s, PROF_PATCH) + PROF_HOST


def tc_lit(nbytes, back):
    """tctx_kernel with an LDS window of nbytes literal bytes from (ls - back) & ~3"""
    return [
        ("  uint8_t qw[kTcQ];\n  uint8_t out[kTx + 4];", "  uint8_t qw[kTcQ];\n  uint8_t lw[%d];\n  uint8_t out[kTx + 4];" % nbytes),
        ("        r.lw = nullptr;\n        r.l_lo = 0;\n        r.l_n = 0;\n        const int j = (int)p0.y;",
         "        const uint32_t lw0 = (h.ls >= %du ? h.ls - %du : 0u) & ~3u;\n"
         "        const PW_GLOBAL uint32_t* l32 = reinterpret_cast<const PW_GLOBAL uint32_t*>((GU8)(A.lits) + lw0);\n"
         "        uint32_t lv[%d];\n#pragma unroll\n        for (int q = 0; q < %d; q++) lv[q] = l32[q];\n"
         "        const int j = (int)p0.y;" % (back, back, nbytes // 4, nbytes // 4)),
        ("        for (int q = 0; q < kTcQ / 16; q++) *reinterpret_cast<LDS v4u*>(me->qw + 16 * q) = qv[q];\n",
         "        for (int q = 0; q < kTcQ / 16; q++) *reinterpret_cast<LDS v4u*>(me->qw + 16 * q) = qv[q];\n"
         "#pragma unroll\n        for (int q = 0; q < %d; q++) reinterpret_cast<LDS uint32_t*>(me->lw)[q] = lv[q];\n"
         "        r.lw = me->lw;\n        r.l_lo = lw0;\n        r.l_n = %du;\n" % (nbytes // 4, nbytes)),
    ]


TC_OPS8 = [("constexpr int kTcOps = 12;", "constexpr int kTcOps = 8;")]


WR_NUM_BF = ("template <class S, int N>\n__device__ __forceinline__ void wr_lit(", """// "%d" of v < 10^8 without the < 10^4 branch (4 digit-pair reads, digits counted by compares)
template <class S>
__device__ __forceinline__ void wr_num_bf(S& k, const LDS SmallTables* t, uint32_t v) {
  if (v >= 100000000u) {
    wr_dig(k, v);
    return;
  }
  const LDS uint16_t* d2 = reinterpret_cast<const LDS uint16_t*>(t->dig2);
  const uint32_t h = v / 10000u, l = v - 10000u * h;
  const uint32_t hh = h / 100u, hl = h - 100u * hh, lh = l / 100u, ll = l - 100u * lh;
  const uint64_t p = (uint64_t)d2[hh] | (uint64_t)d2[hl] << 16 | (uint64_t)d2[lh] << 32 | (uint64_t)d2[ll] << 48;
  const int nd = 1 + (v >= 10u) + (v >= 100u) + (v >= 1000u) + (v >= 10000u) + (v >= 100000u) + (v >= 1000000u) +
                 (v >= 10000000u);
  const uint64_t q = p >> (8 * (8 - nd));
  const uint32_t w[2] = {(uint32_t)q, (uint32_t)(q >> 32)};
  k.put_bytes(w, nd);
}
template <class S, int N>
__device__ __forceinline__ void wr_lit(""")


FX_LDS = [
    ("        f.pad = 0;\n        f.dst = g0;", "        f.pad = (uint32_t)linelen;\n        f.dst = g0;"),
    ("  __shared__ uint32_t ex[kWaves][kWave];  // exclusive prefix of their popcounts\n",
     "  __shared__ uint32_t ex[kWaves][kWave];  // exclusive prefix of their popcounts\n"
     "  __shared__ uint32_t fxb[256][kFxBuf / 4 + 1];\n"),
    ("constexpr int kFxLit = 32;\n", "constexpr int kFxLit = 32;\nconstexpr int kFxBuf = 160;\n"),
    ("""    GlobalSink g;
    g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);
    g.pos = 0;
    int rel;
    emit_event(g, r, in, skip, rel);
""", """    int rel;
    if (f.pad <= (uint32_t)kFxBuf) {
      LDS uint8_t* lb = (LDS uint8_t*)&fxb[threadIdx.x][0];
      LdsSink<kFxBuf> ls;
      ls.buf = lb;
      ls.junk = lb + kFxBuf;
      ls.pos = 0;
      emit_event(ls, r, in, skip, rel);
      PW_GLOBAL uint8_t* d = (PW_GLOBAL uint8_t*)(A.text + f.dst);
      const int n = (int)f.pad;
      int hd = (int)((4u - ((uint32_t)f.dst & 3u)) & 3u);
      if (hd > n) hd = n;
      int i = 0;
      for (; i < hd; i++) d[i] = lb[i];
      for (; i + 4 <= n; i += 4)
        *reinterpret_cast<PW_GLOBAL uint32_t*>(d + i) =
            (uint32_t)lb[i] | ((uint32_t)lb[i + 1] << 8) | ((uint32_t)lb[i + 2] << 16) | ((uint32_t)lb[i + 3] << 24);
      for (; i < n; i++) d[i] = lb[i];
    } else {
      GlobalSink g;
      g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);
      g.pos = 0;
      emit_event(g, r, in, skip, rel);
    }
"""),
]


FX_PAR = [
    ("""    const Fixup f = W.fix[(c0 + (uint64_t)k) * kWave + (uint64_t)__builtin_ctzll(mm)];
    const Hot h = W.hot[f.s];""", """    const uint64_t sl = (c0 + (uint64_t)k) * kWave + (uint64_t)__builtin_ctzll(mm);  // (= f.s)
    const uint64_t fdst = W.fix[sl].dst;
    const Hot h = W.hot[sl];"""),
    ("const Cold cd = W.cold[f.s];", "const Cold cd = W.cold[sl];"),
    ("W.tx + (uint64_t)kTx * f.s);\n      t0 = tp4[0];", "W.tx + (uint64_t)kTx * sl);\n      t0 = tp4[0];"),
    ("g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);", "g.p = (PW_GLOBAL uint8_t*)(A.text + fdst);"),
]


def rev_src(rev):
    return subprocess.run(["git", "show", f"{rev}:pwasm_amd/csrc/pw_report.hip"], cwd=REPO, check=True,
                          capture_output=True, text=True).stdout


def variants():
    """name -> source text; edit this table per experiment (splice(), patched())"""
    cur, head = open(SRC).read(), head_src()
    return {
        "head": head,
        "cur": cur,
        "base3": lambda: rev_src("8ee5aa5"),  # round 3 before the render fast lanes
        "fast3": lambda: rev_src("1c76643"),  # + RecFast
        "fx_lds": lambda: patched(cur, FX_LDS),
        "fx_par": lambda: patched(cur, FX_PAR),
        "r_grid6": lambda: patched(cur, [("if (rg > (uint64_t)ncu * pw::kRenderOcc) rg = (uint64_t)ncu * pw::kRenderOcc;",
                                          "if (rg > (uint64_t)ncu * 6u) rg = (uint64_t)ncu * 6u;")]),
        "r_grid9": lambda: patched(cur, [("rg = (uint64_t)ncu * 2u * pw::kRenderOcc;", "rg = (uint64_t)ncu * 3u * pw::kRenderOcc;")]),
        "r_grid12": lambda: patched(cur, [("rg = (uint64_t)ncu * 2u * pw::kRenderOcc;", "rg = (uint64_t)ncu * 4u * pw::kRenderOcc;")]),
        "ig8": lambda: patched(cur, [("if (ig > (uint64_t)ncu * 10u) ig = (uint64_t)ncu * 10u;", "if (ig > (uint64_t)ncu * 8u) ig = (uint64_t)ncu * 8u;")]),
        "ig12": lambda: patched(cur, [("if (ig > (uint64_t)ncu * 10u) ig = (uint64_t)ncu * 10u;", "if (ig > (uint64_t)ncu * 12u) ig = (uint64_t)ncu * 12u;")]),
        "tg3": lambda: patched(cur, [("if (tg > (uint64_t)ncu * 4u) tg = (uint64_t)ncu * 4u;", "if (tg > (uint64_t)ncu * 3u) tg = (uint64_t)ncu * 3u;")]),
        "tg6": lambda: patched(cur, [("if (tg > (uint64_t)ncu * 4u) tg = (uint64_t)ncu * 4u;", "if (tg > (uint64_t)ncu * 6u) tg = (uint64_t)ncu * 6u;")]),
        "prof": lambda: profiled(cur),
        "tc_small5": lambda: patched(cur, TC_OPS8 + [("constexpr int kTcQ = 48;", "constexpr int kTcQ = 32;"),
                                               ("if (tg > (uint64_t)ncu * 4u) tg = (uint64_t)ncu * 4u;", "if (tg > (uint64_t)ncu * 5u) tg = (uint64_t)ncu * 5u;")]),
        "tc_small6": lambda: patched(cur, TC_OPS8 + [("constexpr int kTcQ = 48;", "constexpr int kTcQ = 32;"),
                                               ("if (tg > (uint64_t)ncu * 4u) tg = (uint64_t)ncu * 4u;", "if (tg > (uint64_t)ncu * 6u) tg = (uint64_t)ncu * 6u;")]),
        "mem": (cur, ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]),
        "num_tloc": lambda: patched(cur, [WR_NUM_BF, ("wr_num(o, r.tab, (uint32_t)(in.tloc + 1));", "wr_num_bf(o, r.tab, (uint32_t)(in.tloc + 1));")]),
        "num_all": lambda: patched(cur, [WR_NUM_BF, ("wr_num(o, r.tab, (uint32_t)(in.tloc + 1));", "wr_num_bf(o, r.tab, (uint32_t)(in.tloc + 1));"),
                                         ("wr_num(o, r.tab, (uint32_t)(e.rloc + 1));", "wr_num_bf(o, r.tab, (uint32_t)(e.rloc + 1));"),
                                         ("wr_num(o, r.tab, (uint32_t)(aap0 + 1));", "wr_num_bf(o, r.tab, (uint32_t)(aap0 + 1));")]),
        "mem_nounroll": (cur, ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause", "-fno-unroll-loops"]),
        "mem_o2": (cur, ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause", "-O2"]),
        "mem_relaxocc": (cur, ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause", "-mllvm", "-amdgpu-schedule-relaxed-occupancy"]),
        "s_maxilp": (cur, ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]),
        "s_maxmem": (cur, ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]),
        "s_iterilp": (cur, ["-mllvm", "-misched=gcn-iterative-ilp"]),
        "s_bias100": (cur, ["-mllvm", "-amdgpu-schedule-metric-bias=100"]),
        "ig5": lambda: patched(cur, [("if (ig > (uint64_t)ncu * 16u) ig = (uint64_t)ncu * 16u;", "if (ig > (uint64_t)ncu * 5u) ig = (uint64_t)ncu * 5u;")]),
        "ig10": lambda: patched(cur, [("if (ig > (uint64_t)ncu * 16u) ig = (uint64_t)ncu * 16u;", "if (ig > (uint64_t)ncu * 10u) ig = (uint64_t)ncu * 10u;")]),
        "ig64": lambda: patched(cur, [("if (ig > (uint64_t)ncu * 16u) ig = (uint64_t)ncu * 16u;", "if (ig > (uint64_t)ncu * 64u) ig = (uint64_t)ncu * 64u;")]),
        "tg8": lambda: patched(cur, [("if (tg > (uint64_t)ncu * 4u) tg = (uint64_t)ncu * 4u;", "if (tg > (uint64_t)ncu * 16u) tg = (uint64_t)ncu * 16u;")]),
        "tc_lit32": lambda: patched(cur, tc_lit(32, 12)),
        "tc_lit16_ops8": lambda: patched(cur, tc_lit(16, 8) + TC_OPS8),
        "tc_ops8": lambda: patched(cur, TC_OPS8),
        "fastcnt": lambda: patched(cur, FASTCNT_PATCH) + PROF_HOST,
        # timing only (parity fails): fixup_kernel without its long lines / without emit_event /
        # without the finalize part
        "fx_nolong": lambda: patched(cur, [("  if (W.ctr[2]) return;  // overflow", "  return;  // overflow")]),
        "fx_noemit": lambda: patched(cur, [("    int rel;\n    emit_event(g, r, in, skip, rel);\n  }",
                                            "    g.p[0] = (uint8_t)(in.tx[0] + me->qw[0] + me->lw[0] + (uint32_t)in.n);\n  }")]),
        "fx_nofin": lambda: patched(cur, [("    if (ai < A.n_alns) finalize_record(A, W, ai);\n    return;", "    return;")]),
        # tctx grid: workgroups per CU (4 resident): 2, 8 (two rounds), 12
        "tg2": lambda: patched(cur, [(TG, TG.replace("4u", "2u"))]),
        "tg8": lambda: patched(cur, [(TG, TG.replace("4u", "8u"))]),
        "tg12": lambda: patched(cur, [(TG, TG.replace("4u", "12u"))]),
    }


def main(names):
    vs = variants()
    objs = [os.path.join(REPO, "pwasm_amd/build", f) for f in sorted(os.listdir(os.path.join(REPO, "pwasm_amd/build")))
            if f.endswith(".o") and f != "pw_report.o"]
    for name in names or list(vs):
        d = os.path.join(OUT, name)
        os.makedirs(os.path.join(d, "lib"), exist_ok=True)
        hip = os.path.join(d, "pw_report.hip")
        v = vs[name]
        extra = ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]  # (as the Makefile builds pw_report)
        if isinstance(v, tuple):
            v, extra = v[0], extra + [f for f in v[1] if f not in extra]
        open(hip, "w").write(v() if callable(v) else v)
        o = os.path.join(d, "pw_report.o")
        inc = ["-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "pwasm_amd/csrc")]
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall",
                        "-Wno-unused-function", *extra, *inc, "-c", hip, "-o", o], check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                        os.path.join(d, "lib", "libpwasm_amd.so"), o, *objs, "-ldl"], check=True)
        print("built", name, flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
