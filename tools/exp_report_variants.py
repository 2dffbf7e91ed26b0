"""Experiment variants of pw_report.hip (never shipped; timing only unless noted) linked into
tools/abl_build/<name>/lib for tools/exp_sweep.sh (PWASM_LIB):
  cur      the working copy
  head     pw_report.hip at git HEAD
  tg8..tg16  tctx_kernel grid of 8 / 12 / 16 workgroups per CU (product: 4)
  ig15..ig30 index_kernel grid of 15 / 20 / 30 workgroups per CU (product: 10)
  rr4 / rr8  render grid of 4 / 8 rounds of resident workgroups (product: 2)
  igp20      index_kernel grid of 20 per CU for long-record (planned) batches (product: 10)
  ns256 / ns1024 next-stop table grid capped at 256 / 1024 workgroups (product: 4096)
  cg4 / cg16 carry_kernel grid of 4 / 16 per CU (product: 8)
  pg4..pg16  index_pair_kernel grid (pg10: the pre-round-4-end 10) of 4 / 8 / 12 / 16 workgroups per CU (product: 10)
  allgen   every render wave takes the general emit_event path (same bytes)
  allfast  every render wave takes emit_fast (wrong bytes where a lane is not fast: timing only)
  noline   no line is built (every line 78 bytes of whatever the buffer holds: timing only)
  nowin    the per-lane query window is not loaded (constant bytes: timing only)
  nohot    the Hot records are replaced by synthetic insertions after the load (timing only)
  nocopy   render's copy-out (LDS page image + stores) skipped (timing only)
  fx_inline  fixup_kernel reads outside its windows inline (no out-of-line call per byte)
  fx_bigwin  fixup_kernel stages 128 query bytes and 64 literal bytes per line
  tc_nowalk  tctx_kernel skips the op walk (timing only)
  rw2      render_kernel in 2-wave workgroups (6 per CU)
  idx_scalar index_kernel record heads through scalar loads
  why      render counts its non-fast lanes by reason into Work.ctr[8..15] (ctr[7]: general waves)
  tw2      tctx_kernel in 2-wave workgroups (8 per CU)
  ls148    148-byte line buffer stride (odd dword count: fewer LDS bank conflicts between lanes)
  h32      32-byte event records whatever the batch (the pre-round-5 format; same bytes)
  qalias / occ4 / occ4q  render's query windows in the line buffers' tails (LDS for 4 workgroups
           per CU) / the 4-per-CU register budget / both (timing only)
  kl108    lines up to 108 bytes built in render (kLine 92 -> 108: the whole 40-byte slack of the
           148-byte stride; copy-out over 28 dwords / 7 groups), so fewer lines go to fixup_kernel
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
    "tc_nowalk": [("      emit_tctx_walk(ks, r, wd >> 30, ne, (uint32_t)j, wd, cd.qs, cd.ts, h.ls);",
                   "      if (A.n_alns == 0) emit_tctx_walk(ks, r, wd >> 30, ne, (uint32_t)j, wd, cd.qs, cd.ts, h.ls);\n      else ks.pos = 11;")],
    # render_kernel in 2-wave workgroups, 6 per CU (same 3 waves/SIMD; a workgroup's LDS frees
    # when its slower wave ends, so smaller workgroups pack the CU more tightly)
    "rw2": [("constexpr int kRenderOcc = 3;   // render_kernel: workgroups per CU (LDS-limited)",
             "constexpr int kRenderOcc = 6;   // render_kernel: workgroups per CU (LDS-limited)\nconstexpr int kRenderWaves = 2;"),
            ("__global__ __launch_bounds__(kWave* kWaves, kRenderOcc) void render_kernel(pw_report_args A, Work W) {\n  __shared__ SmallTables tab;\n  __shared__ __attribute__((aligned(16))) RenderWave rw[kWaves];\n  LDS SmallTables* tp = (LDS SmallTables*)&tab;\n  stage_small_tables(tp, threadIdx.x, kWave * kWaves);",
             "__global__ __launch_bounds__(kWave* kRenderWaves, 3) void render_kernel(pw_report_args A, Work W) {\n  __shared__ SmallTables tab;\n  __shared__ __attribute__((aligned(16))) RenderWave rw[kRenderWaves];\n  LDS SmallTables* tp = (LDS SmallTables*)&tab;\n  stage_small_tables(tp, threadIdx.x, kWave * kRenderWaves);"),
            ("  const uint64_t nw = (uint64_t)gridDim.x * kWaves;\n\n  uint64_t c = (uint64_t)blockIdx.x * kWaves + wv;\n  if (c >= W.n_chunks) return;\n  Hot h = decode_hot(load_hot(W, c, lane), true);",
             "  const uint64_t nw = (uint64_t)gridDim.x * kRenderWaves;\n\n  uint64_t c = (uint64_t)blockIdx.x * kRenderWaves + wv;\n  if (c >= W.n_chunks) return;\n  Hot h = decode_hot(load_hot(W, c, lane), true);"),
            ("    uint64_t rg = (W.n_chunks + nwave - 1) / nwave;", "    uint64_t rg = (W.n_chunks + pw::kRenderWaves - 1) / pw::kRenderWaves;"),
            ("    hipLaunchKernelGGL(pw::render_kernel, dim3((uint32_t)rg), dim3(pw::kWave * pw::kWaves), 0, st, *args, W);",
             "    hipLaunchKernelGGL(pw::render_kernel, dim3((uint32_t)rg), dim3(pw::kWave * pw::kRenderWaves), 0, st, *args, W);")],
    # tctx_kernel in 2-wave workgroups, 8 per CU (same 4 waves/SIMD, finer packing)
    "tw2": [("__global__ __launch_bounds__(kWave* kWaves) void tctx_kernel(pw_report_args A, Work W) {",
             "constexpr int kTctxWaves = 2;\n__global__ __launch_bounds__(kWave* kTctxWaves) void tctx_kernel(pw_report_args A, Work W) {"),
            ("  __shared__ __attribute__((aligned(16))) TctxWave tw[kWaves];", "  __shared__ __attribute__((aligned(16))) TctxWave tw[kTctxWaves];"),
            ("  stage_small_tables(tp, threadIdx.x, kWave * kWaves);\n  __syncthreads();\n  const int lane = threadIdx.x & (kWave - 1), wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);\n  LDS TctxWave* w",
             "  stage_small_tables(tp, threadIdx.x, kWave * kTctxWaves);\n  __syncthreads();\n  const int lane = threadIdx.x & (kWave - 1), wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);\n  LDS TctxWave* w"),
            ("  const uint64_t gstride = (uint64_t)gridDim.x * kWaves;\n  uint64_t gi = (uint64_t)blockIdx.x * kWaves + wv;",
             "  const uint64_t gstride = (uint64_t)gridDim.x * kTctxWaves;\n  uint64_t gi = (uint64_t)blockIdx.x * kTctxWaves + wv;"),
            ("    uint64_t tg = (W.n_chunks * pw::kWave + 255) / 256 / pw::kWaves + 1;\n    if (tg > (uint64_t)ncu * 4u) tg = (uint64_t)ncu * 4u;\n    hipLaunchKernelGGL(pw::tctx_kernel, dim3((uint32_t)tg), dim3(pw::kWave * pw::kWaves), 0, st, *args, W);",
             "    uint64_t tg = (W.n_chunks * pw::kWave + 255) / 256 / pw::kTctxWaves + 1;\n    if (tg > (uint64_t)ncu * 8u) tg = (uint64_t)ncu * 8u;\n    hipLaunchKernelGGL(pw::tctx_kernel, dim3((uint32_t)tg), dim3(pw::kWave * pw::kTctxWaves), 0, st, *args, W);")],
    # index_kernel: the record heads (descriptor, query location, next event slot) as scalar loads
    # instead of per-lane vector loads pinned in VGPRs
    "idx_scalar": [('  asm volatile("" : "+v"(p.qb), "+v"(p.ev_next), "+v"(p.L), "+v"(p.w0), "+v"(p.w1));',
                    '  asm volatile("" : "+v"(p.w0), "+v"(p.w1));'),
                   ("    rec_pre_ready(A, cur, lane);\n    pin(dn.a);\n    pin(dn.b);", "    rec_pre_ready(A, cur, lane);"),
                   ("      rec_pre_ready(A, nxt, lane);\n      pin(dnn.a);\n      pin(dnn.b);", "      rec_pre_ready(A, nxt, lane);")],
    # render: why lanes miss the fast path — per reason an atomic into Work.ctr[8..14] (bench logs
    # ctr[8:16]; timing meaningless)
    "why": [("      int merr;\n      if (__ballot(!fast) == 0) {",
             "      if (!fast) {\n        const int why = !r.acgt ? 8 : (rlc < 8 ? 9 : ((r.L >= 100000000 || hc.tloc >= 99999999) ? 10 : "
             "(typ == PW_OP_SUB ? (n > 4 ? 11 : 12) : (typ == PW_OP_INS ? (n > 8 ? 13 : 14) : 15))));\n"
             "        atomicAdd(&W.ctr[why], 1u);\n      }\n      if (__ballot(!fast) != 0 && lane == 0) atomicAdd(&W.ctr[7], 1u);\n"
             "      int merr;\n      if (__ballot(!fast) == 0) {")],
    # fixup_kernel's two halves timed apart (results wrong: timing only)
    "fx_nofin": [("    if (ai < A.n_alns) finalize_record(A, W, ai);\n    return;", "    return;")],
    "fx_nofix": [("  if (W.ctr[2]) return;  // overflow: the results report it, nothing is rewritten", "  return;")],
    # finalize as its own launch before the (then long-line only) fixup launch
    "fx_sep": [("    if (ai < A.n_alns) finalize_record(A, W, ai);\n    return;", "    return;"),
               ("    hipLaunchKernelGGL(pw::fixup_kernel, dim3(",
                "    hipLaunchKernelGGL(pw::finalize_kernel, dim3((uint32_t)((args->n_alns + 255) / 256)), dim3(256), 0, st, *args, W);\n"
                "    hipLaunchKernelGGL(pw::fixup_kernel, dim3(")],
    "fx_lds": [("  __shared__ __attribute__((aligned(16))) FixLane fl[256];", "  __shared__ __attribute__((aligned(16))) FixLane fl[4];"),
               ("  LDS FixLane* me = (LDS FixLane*)&fl[threadIdx.x];", "  LDS FixLane* me = (LDS FixLane*)&fl[threadIdx.x & 3];")],
    "fx_sep2": [("    if (ai < A.n_alns) finalize_record(A, W, ai);\n    return;", "    return;"),
                ("    hipLaunchKernelGGL(pw::fixup_kernel, dim3((uint32_t)ncu + (uint32_t)((args->n_alns + 255) / 256)), dim3(256), 0,",
                 "    hipLaunchKernelGGL(pw::finalize_kernel, dim3((uint32_t)((args->n_alns + 255) / 256)), dim3(256), 0, st, *args, W);\n"
                 "    hipLaunchKernelGGL(pw::fixup_kernel, dim3((uint32_t)ncu), dim3(256), 0,"),
                ("  const uint32_t fix_wg = gridDim.x - (A.n_alns + 255) / 256;", "  const uint32_t fix_wg = gridDim.x;")],
    # fixup_kernel timed on the long lines render's fast predicate accepts / rejects only
    "fx_onlyfast": [("    GlobalSink g;\n    g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);",
                     "    const bool fast_ = r.acgt && rl >= 4 && r.L >= 9 && r.L < 100000000 && h.tloc < 99999999 && (typ == PW_OP_SUB ? (ne <= 4 && 3 * (rl / 3 - 1) + 9 <= r.L) : ne <= (typ == PW_OP_INS ? 8 : 12));\n    if (!fast_) continue;\n    GlobalSink g;\n    g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);")],
    "fx_onlyslow": [("    GlobalSink g;\n    g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);",
                     "    const bool fast_ = r.acgt && rl >= 4 && r.L >= 9 && r.L < 100000000 && h.tloc < 99999999 && (typ == PW_OP_SUB ? (ne <= 4 && 3 * (rl / 3 - 1) + 9 <= r.L) : ne <= (typ == PW_OP_INS ? 8 : 12));\n    if (fast_) continue;\n    GlobalSink g;\n    g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);")],
    # fixup_kernel's long-line chain timed in stages (s_memtime after full waits): ctr[7] whole line,
    # [8] mask -> Fixup -> Hot, [9] windows staged, [10] emit_event, [11] lines on one lane (maxima)
    "fx_time": [("    const Fixup f = W.fix[(c0 + (uint64_t)k) * kWave + (uint64_t)__builtin_ctzll(mm)];",
                 "    __builtin_amdgcn_s_waitcnt(0);\n    const uint64_t TA = clock64();\n"
                 "    const Fixup f = W.fix[(c0 + (uint64_t)k) * kWave + (uint64_t)__builtin_ctzll(mm)];"),
                ("    const int rl = event_rloc(r.L, rev, typ, h.qp, ne);\n    int x0 = rl - 8;\n    if (x0 < 0) x0 = 0;\n    const int x0a = x0 & ~15;  // (r.R is 16-byte aligned)\n    const GV4* a0",
                 "    __builtin_amdgcn_s_waitcnt(0);\n    const uint64_t TB = clock64();\n"
                 "    const int rl = event_rloc(r.L, rev, typ, h.qp, ne);\n    int x0 = rl - 8;\n    if (x0 < 0) x0 = 0;\n    const int x0a = x0 & ~15;  // (r.R is 16-byte aligned)\n    const GV4* a0"),
                ("    GlobalSink g;\n    g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);",
                 "    __builtin_amdgcn_s_waitcnt(0);\n    const uint64_t TC = clock64();\n"
                 "    GlobalSink g;\n    g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);"),
                ("    emit_event(g, r, in, skip, rel);\n  }",
                 "    emit_event(g, r, in, skip, rel);\n    __builtin_amdgcn_s_waitcnt(0);\n    const uint64_t TD = clock64();\n"
                 "    atomicMax(&W.ctr[7], (uint32_t)(TD - TA));\n    atomicMax(&W.ctr[8], (uint32_t)(TB - TA));\n"
                 "    atomicMax(&W.ctr[9], (uint32_t)(TC - TB));\n    atomicMax(&W.ctr[10], (uint32_t)(TD - TC));\n"
                 "    atomicMax(&W.ctr[11], (T + 63u - (uint32_t)lane) / 64u);\n  }")],
    # fixup_kernel launched twice per pass (idempotent): is the second, warm-cache launch faster?
    "fx_twice": [("    hipLaunchKernelGGL(pw::fixup_kernel, dim3((uint32_t)ncu + (uint32_t)((args->n_alns + 255) / 256)), dim3(256), 0,\n                       st, *args, W);",
                  "    hipLaunchKernelGGL(pw::fixup_kernel, dim3((uint32_t)ncu + (uint32_t)((args->n_alns + 255) / 256)), dim3(256), 0,\n                       st, *args, W);\n"
                  "    hipLaunchKernelGGL(pw::fixup_kernel, dim3((uint32_t)ncu + (uint32_t)((args->n_alns + 255) / 256)), dim3(256), 0,\n                       st, *args, W);")],
    # no next-stop table build (timing only: index without the side-stream kernel beside it)
    "ns_skip": [("  const uint32_t grid = nq < 4096u ? nq : 4096u;\n  hipLaunchKernelGGL(pw::stop_table_kernel,",
                 "  const uint32_t grid = nq < 4096u ? nq : 4096u;\n  if (grid) return PW_OK;\n  hipLaunchKernelGGL(pw::stop_table_kernel,")],
    # index_kernel at 6 waves/SIMD (<= 80 VGPRs), grid two rounds of that
    "idx6": [("constexpr int kIndexOcc = 5;", "constexpr int kIndexOcc = 6;"),
             ("  if (ig > (uint64_t)ncu * 10u || planned) ig = (uint64_t)ncu * 10u;",
              "  if (ig > (uint64_t)ncu * 12u || planned) ig = (uint64_t)ncu * 12u;")],
    "idx6g10": [("constexpr int kIndexOcc = 5;", "constexpr int kIndexOcc = 6;")],
    # no counter memset before index (timing only: cfg2 uses no counter that carries over harmfully)
    "nomemset": [("  if (hipMemsetAsync(args->workspace, 0, 64, st) != hipSuccess) return PW_E_HIP;", "")],
    # the same source under other machine schedulers (FLAGS below)
    "sch_ilp": [],
    "sch_none": [],
    "sch_iterilp": [],
    "sch_minreg": [],
    # fixup_kernel: the Hot / Cold / tx records by the line's slot (the lane-mask position) in
    # parallel with its Fixup entry, whose `s` is the same slot (one dependent load less per line)
    "fx_par": [("    const Fixup f = W.fix[(c0 + (uint64_t)k) * kWave + (uint64_t)__builtin_ctzll(mm)];\n    const Hot h = W.hot[f.s];",
                "    const uint64_t sl = (c0 + (uint64_t)k) * kWave + (uint64_t)__builtin_ctzll(mm);  // (= f.s)\n"
                "    const uint64_t fdst = W.fix[sl].dst;\n    const Hot h = W.hot[sl];"),
               ("const Cold cd = W.cold[f.s];", "const Cold cd = W.cold[sl];"),
               ("W.tx + (uint64_t)kTx * f.s);\n      t0 = tp4[0];", "W.tx + (uint64_t)kTx * sl);\n      t0 = tp4[0];"),
               ("g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);", "g.p = (PW_GLOBAL uint8_t*)(A.text + fdst);")],
    "fx_bigwin": [("constexpr int kFxLit = 32;", "constexpr int kFxLit = 64;\nconstexpr int kFxQ = 128;"),
                  ("  uint8_t qw[kQWin];\n  uint8_t lw[kFxLit];", "  uint8_t qw[kFxQ];\n  uint8_t lw[kFxLit];"),
                  ("    for (int q = 0; q < kQWin / 16; q++) *reinterpret_cast<LDS v4u*>(me->qw + 16 * q) = a0[q];",
                   "    for (int q = 0; q < kFxQ / 16; q++) *reinterpret_cast<LDS v4u*>(me->qw + 16 * q) = a0[q];"),
                  ("    r.qw = me->qw;\n    r.qlo = x0a;\n    r.qn = kQWin;", "    r.qw = me->qw;\n    r.qlo = x0a;\n    r.qn = kFxQ;")],
    "kl108": [("constexpr int kLine = 92; ", "constexpr int kLine = 108;"),
              ("      uint32_t Lw[24];", "      uint32_t Lw[28];"),
              ("        for (int q = 0; q < 6; q++) {\n          const v4u v = lp4[q];",
               "        for (int q = 0; q < 7; q++) {\n          const v4u v = lp4[q];"),
              ("          const uint32_t cur = k < 24 ? Lw[k] : 0u,", "          const uint32_t cur = k < 28 ? Lw[k] : 0u,"),
              ("        for (int j = 5; j >= 0; j--)\n          if (j <= jmax) *reinterpret_cast<LDS v4a4*>",
               "        for (int j = 6; j >= 0; j--)\n          if (j <= jmax) *reinterpret_cast<LDS v4a4*>"),
              ("        for (int j = 5; j >= 0; j--)\n          __builtin_amdgcn_raw_buffer_store_b128(group(j)",
               "        for (int j = 6; j >= 0; j--)\n          __builtin_amdgcn_raw_buffer_store_b128(group(j)")],
}

# index_pair_kernel grid (workgroups per CU; the product's 10 was swept for index_kernel at 5
# waves/SIMD, the pair kernel runs at 4)
for _g in (4, 10, 12, 16):  # (the product took 8 in round 4)
    PATCHES[f"pg{_g}"] = [("nwave - 1) / nwave, (uint64_t)ncu * 8u)),", f"nwave - 1) / nwave, (uint64_t)ncu * {_g}u)),")]
# tctx_kernel grid (workgroups per CU; product 4) and index_kernel grid (product 10)
for _g in (8, 12, 16):
    PATCHES[f"tg{_g}"] = [("if (tg > (uint64_t)ncu * 4u) tg = (uint64_t)ncu * 4u;", f"if (tg > (uint64_t)ncu * {_g}u) tg = (uint64_t)ncu * {_g}u;")]
for _g in (15, 20, 30):
    PATCHES[f"ig{_g}"] = [("if (ig > (uint64_t)ncu * 10u || planned) ig = (uint64_t)ncu * 10u;",
                           f"if (ig > (uint64_t)ncu * {_g}u || planned) ig = (uint64_t)ncu * {_g}u;")]
# render grid in rounds of the resident workgroups (product: 2), long-record (planned) index grid
# and carry_kernel grid (product: 10 / 8 per CU)
for _g in (4, 8):
    PATCHES[f"rr{_g}"] = [("if (rg > (uint64_t)ncu * 2u * pw::kRenderOcc) rg = (uint64_t)ncu * 2u * pw::kRenderOcc;",
                           f"if (rg > (uint64_t)ncu * {_g}u * pw::kRenderOcc) rg = (uint64_t)ncu * {_g}u * pw::kRenderOcc;")]
PATCHES["igp20"] = [("if (planned) ig = (uint64_t)ncu * 10u;", "if (planned) ig = (uint64_t)ncu * 20u;")]
PATCHES["cg16"] = [("pw::carry_kernel, dim3((uint32_t)ncu * 8u)", "pw::carry_kernel, dim3((uint32_t)ncu * 16u)")]
PATCHES["cg4"] = [("pw::carry_kernel, dim3((uint32_t)ncu * 8u)", "pw::carry_kernel, dim3((uint32_t)ncu * 4u)")]
# next-stop table grid (product: min(queries, 4096) workgroups, one query each at a time)
for _g in (256, 1024):
    PATCHES[f"ns{_g}"] = [("  const uint32_t grid = nq < 4096u ? nq : 4096u;", f"  const uint32_t grid = nq < {_g}u ? nq : {_g}u;")]
PATCHES["fx_pb"] = PATCHES["fx_par"] + PATCHES["fx_bigwin"]  # (both)
# 32-byte event records whatever the batch (round 5: 16-byte records when the queries fit)
PATCHES["h32"] = [("  W.hot_pbits = args->hot_pbits;\n  W.hot_sh = args->hot_pbits ? 2u : 3u;",
                   "  W.hot_pbits = 0;\n  W.hot_sh = 3u;")]

# render occupancy (round 5, timing only): the query windows placed in the line buffers' tails
# (bytes 100-147 of each lane's 148-byte buffer: 37.9 KB of LDS per workgroup, room for 4 per CU;
# a line past 100 bytes overwrites its own window), with / without the 4-per-CU register budget
# (128 VGPRs: hipcc spills the rest)
_QALIAS = [("  uint8_t qw[kWave * kQStride];     // per-lane forward-query windows\n", ""),
           ("  LDS uint8_t* my_qw = w->qw + lane * kQStride;", "  LDS uint8_t* my_qw = w->line + lane * kLStride + 100;")]
PATCHES["qalias"] = _QALIAS
PATCHES["occ4"] = [("constexpr int kRenderOcc = 3;", "constexpr int kRenderOcc = 4;")]
PATCHES["occ4q"] = _QALIAS + PATCHES["occ4"]

# (the same with the window stored as dwords: 8-byte stores at the 4-byte aligned tails replay)
_QALIAS2 = _QALIAS + [("""      *reinterpret_cast<LDS v2u*>(my_qw + 16 * q) = (v2u){pre.q[q].x, pre.q[q].y};
      *reinterpret_cast<LDS v2u*>(my_qw + 16 * q + 8) = (v2u){pre.q[q].z, pre.q[q].w};""",
                      """      {
        volatile LDS uint32_t* q4 = reinterpret_cast<volatile LDS uint32_t*>(my_qw + 16 * q);
        q4[0] = pre.q[q].x;
        q4[1] = pre.q[q].y;
        q4[2] = pre.q[q].z;
        q4[3] = pre.q[q].w;
      }""")]
PATCHES["qalias2"] = _QALIAS2
PATCHES["occ4q2"] = _QALIAS2 + PATCHES["occ4"]

# index_kernel at 4 waves/SIMD (128 VGPRs; product: 5)
PATCHES["idx4"] = [("constexpr int kIndexOcc = 5;", "constexpr int kIndexOcc = 4;")]

# render with the next chunk's inputs issued before this chunk's line is built (one whole
# iteration of lead instead of the copy-out's): the Hot records three chunks ahead, the query
# starts two ahead (round 5, timing + register experiment)
PATCHES["early"] = [
    ("""  HotRaw<kH16> hn = load_hot<kH16>(W, c + nw, lane);
  RenderPre pre;
  render_pre<kH16>(A, W, h, c * kWave + (uint64_t)lane, skip, pre);""",
     """  HotRaw<kH16> hn = load_hot<kH16>(W, c + nw, lane);
  if constexpr (kH16) qn = load_qinfo(A, W, hn);
  HotRaw<kH16> hn2 = load_hot<kH16>(W, c + 2 * nw, lane);
  RenderPre pre;
  render_pre<kH16>(A, W, h, c * kWave + (uint64_t)lane, skip, pre);"""),
    ("""    render_pre_ready<kH16>(pre);
    if constexpr (kH16) {
      // the next chunk's query starts / lengths (its records came in with this chunk's inputs),
      // consumed when it is decoded after this chunk's lines; this chunk's first literal bytes
      qn = load_qinfo(A, W, hn);
      lit8(h.ls, pre.lw[0], pre.lw[1], pre.lw[2], h.l0, h.l1);
    }""",
     """    render_pre_ready<kH16>(pre);
    if constexpr (kH16) lit8(h.ls, pre.lw[0], pre.lw[1], pre.lw[2], h.l0, h.l1);"""),
    ("""    const v4u t0 = pre.t0, t1 = pre.t1;
    const int ns_pre = pre.ns_ok ? (int)pre.ns_raw : kNsNone;
    const int qlo = pre.qlo, n_cur = pre.n;""",
     """    const v4u t0 = pre.t0, t1 = pre.t1;
    const int ns_pre = pre.ns_ok ? (int)pre.ns_raw : kNsNone;
    const int qlo = pre.qlo, n_cur = pre.n;
    const uint32_t ai_cur = pre.ai;
    // the next chunk: decoded and its inputs issued now, in flight during this chunk's line
    if constexpr (kH16) pin(qn);
    const Hot hx = decode_hot<kH16>(W, hn, qn, c + nw < W.n_chunks);
    render_pre<kH16>(A, W, hx, (c + nw) * kWave + (uint64_t)lane, skip, pre);
    if constexpr (kH16) qn = load_qinfo(A, W, hn2);
    hn = hn2;
    hn2 = load_hot<kH16>(W, c + 3 * nw, lane);"""),
    ("""    const uint32_t fn_cur = h.fn;
    const uint32_t ai_cur = pre.ai;
    // the next chunk's inputs load behind this one's output
    if constexpr (kH16) pin(qn);
    h = decode_hot<kH16>(W, hn, qn, c + nw < W.n_chunks);
    hn = load_hot<kH16>(W, c + 2 * nw, lane);
    render_pre<kH16>(A, W, h, (c + nw) * kWave + (uint64_t)lane, skip, pre);""",
     """    const uint32_t fn_cur = h.fn;
    h = hx;"""),
]

PATCHES["early2"] = PATCHES["early"] + [("constexpr int kRenderOcc = 3;", "constexpr int kRenderOcc = 2;")]

# render's text stores with a cache policy (round 5): nt (aux 2) or sc1 (aux 16: write-through,
# the line leaves the XCD's L2 — the text is never read again on the GPU)
for _nm, _aux in (("txt_nt", 2), ("txt_sc1", 16)):
    PATCHES[_nm] = [
        ("__builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const LDS v4u*>(img + o), rs, o < B ? o : kDropOff, 0, 0);",
         f"__builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const LDS v4u*>(img + o), rs, o < B ? o : kDropOff, 0, {_aux});"),
        ("__builtin_amdgcn_raw_buffer_store_b128(group(j), rs, j <= jmax ? a0 + 16u * (uint32_t)j : kDropOff, 0, 0);",
         f"__builtin_amdgcn_raw_buffer_store_b128(group(j), rs, j <= jmax ? a0 + 16u * (uint32_t)j : kDropOff, 0, {_aux});")]

# non-temporal stores of index's 16-byte event records / tctx's tx records (round 5)
PATCHES["hot_nt"] = [("    p[0] = (v4u){h.fn, qi << W.hot_pbits | (uint32_t)h.qp, (uint32_t)h.tloc, h.ls};",
                      "    __builtin_nontemporal_store((v4u){h.fn, qi << W.hot_pbits | (uint32_t)h.qp, (uint32_t)h.tloc, h.ls}, p);")]
PATCHES["tx_nt"] = [("      dtx[0] = t0;\n      dtx[1] = t1;", "      __builtin_nontemporal_store(t0, dtx);\n      __builtin_nontemporal_store(t1, dtx + 1);")]

# index's op-word loads non-temporal (a once-read stream for index)
PATCHES["ops_nt"] = [
    ("  p.w0 = *((uint32_t)lane < d.n_ops ? ops + lane : dummy);\n  p.w1 = *((uint32_t)(lane + 64) < d.n_ops ? ops + lane + 64 : dummy);",
     "  p.w0 = __builtin_nontemporal_load((uint32_t)lane < d.n_ops ? ops + lane : dummy);\n  p.w1 = __builtin_nontemporal_load((uint32_t)(lane + 64) < d.n_ops ? ops + lane + 64 : dummy);"),
    ("        uint32_t w = ops[idx < nseg ? sb + idx : sb];", "        uint32_t w = __builtin_nontemporal_load(ops + (idx < nseg ? sb + idx : sb));")]

# render's Hot record loads / tx loads non-temporal (round 5)
PATCHES["hotld_nt"] = [("  r.a = p[0];\n  if constexpr (!kH16) r.b = p[1];",
                        "  r.a = __builtin_nontemporal_load(p);\n  if constexpr (!kH16) r.b = __builtin_nontemporal_load(p + 1);")]
PATCHES["txld_nt"] = [("    p.t0 = tp4[0];\n    p.t1 = tp4[1];", "    p.t0 = __builtin_nontemporal_load(tp4);\n    p.t1 = __builtin_nontemporal_load(tp4 + 1);")]

# fixup_kernel's long lines emitted into one shared LDS scratch line instead of global memory (no
# global byte stores: wrong output, timing only)
PATCHES["fx_ldssink"] = [("""    GlobalSink g;
    g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);
    g.pos = 0;
    int rel;
    emit_event(g, r, in, skip, rel);""", """    LdsSink<128> g;
    g.buf = (LDS uint8_t*)&lsk[0];
    g.junk = g.buf + 128;
    g.pos = 0;
    int rel;
    emit_event(g, r, in, skip, rel);
    if (g.pos == 12345) A.text[f.dst] = 0;"""),
    ("  __shared__ uint32_t ex[kWaves][kWave];  // exclusive prefix of their popcounts",
     "  __shared__ uint32_t ex[kWaves][kWave];  // exclusive prefix of their popcounts\n  __shared__ uint8_t lsk[136];")]

# render's long-line epilogue (round 5): left out (listed lines never written: timing only), or
# compiled in but never run
PATCHES["le_none"] = [("  if (n_long > 0) {  // (the lane-derived", "  if (n_long > 0 && A.n_alns == 0xFFFFFFFFu) {  // (the lane-derived"),
                      ("__device__ __forceinline__ void render_long_lines(", "__device__ __forceinline__ void render_long_lines_x(const int);\n__device__ __forceinline__ void render_long_lines(")]
PATCHES["le_cold"] = [("  if (n_long > 0) {  // (the lane-derived", "  if (n_long > 0 && A.n_alns == 0xFFFFFFFFu) {  // (the lane-derived")]
PATCHES["le_skip"] = [("  if (n_long > 0) {  // (the lane-derived", "  if (false) {  // (the lane-derived")]

# timing only (wrong bytes): the walk's byte reads outside the staged windows / literal registers
# answered without their global load
PATCHES["nolitg"] = [("  return lit_global(r.lits, i);\n}", "  return r.lits == nullptr ? lit_global(r.lits, i) : (uint8_t)'A';\n}")]
PATCHES["norcg"] = [("  if (o < (unsigned)r.qn) return r.qw[o];\n  return rc_global(r.R, r.L, x);",
                     "  if (o < (unsigned)r.qn) return r.qw[o];\n  return r.R == nullptr ? rc_global(r.R, r.L, x) : (uint8_t)'A';")]

# scheduler flags per variant (default: the Makefile's max-memory-clause)
FLAGS = {
    "sch_ilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "sch_none": [],
    "sch_iterilp": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
    "sch_minreg": ["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"],
}


def build(name):
    s = open(SRC).read()
    if "=" in name:  # name=path: a saved copy of pw_report.hip built as variant `name`
        name, path = name.split("=", 1)
        s = open(path).read()
    elif name == "head":  # pw_report.hip as committed at git HEAD (the A of an A/B against an uncommitted edit)
        s = subprocess.run(["git", "-C", REPO, "show", "HEAD:pwasm_amd/csrc/pw_report.hip"], check=True,
                           capture_output=True, text=True).stdout
    for a, b in PATCHES.get(name, []):
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
                    "-Wno-unused-function", *FLAGS.get(name, ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]), *inc, "-c", src,
                    "-o", o], check=True)
    bdir = os.path.join(REPO, "pwasm_amd/build")
    objs = [os.path.join(bdir, f) for f in sorted(os.listdir(bdir)) if f.endswith(".o") and f != "pw_report.o"]
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                    os.path.join(d, "lib", "libpwasm_amd.so"), o, *objs, "-ldl"], check=True)
    print("built", name, flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(PATCHES):
        build(n)
