"""Experiment variants of pw_msa.hip for attributing tile_counts' time and LDS bank conflicts
(never shipped; timing only — the counting variants give wrong counts, parity FAILs by design):
  cur      the product source
  noflush  the LDS counter-table flush (cnt_flush) never runs (counters still accumulated)
  nowin    the row window is not stored to LDS (loads kept, reads see a stale window)
  noruns   the gap-run ORs into the bitmap are skipped
  rp_lds   profiles/variants/row_prefix_lds.patch (row_prefix stages the row's runs in LDS)
  k1_3ahead  row_chunk_sums with three groups' loads in flight instead of two
  k1_32b   profiles/variants/row_chunk_sums_32bases.patch (8 lanes x 32 bases per chunk)
  k1g<N>   row_chunk_sums with a grid of N workgroups (product: 2048)
  sy<N>    slot_rows with N workgroups per row (product: 2048 / rows)
  nogather no window reads at all (the group bytes a constant: the cost of the LDS gather)
  (round 5, measured then dropped from this list: idealsrc — reads at the gap-free offsets,
  norot — no per-lane rotation of the column groups (adopted), runs2 — gap-run ORs as two
  words + a loop past 33 columns (93.7 vs 90.5 us))
  rowlist8 / rowlist8mid  tile_counts_rowlist16.patch at 8 waves per workgroup (rows that meet the
           tile listed and shared equally; mid: tiles from the middle outwards)
  head     pw_msa.hip as committed at git HEAD (the A of an A/B against an uncommitted edit)
Usage: python tools/exp_msa_variants.py [names...]  -> tools/abl_build/<name>/lib (tools/exp_msa.py)"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "pwasm_amd/csrc/pw_msa.hip")
TMP = os.path.join(REPO, "build_exp")


def sub(s, old, new):
    assert old in s, old
    return s.replace(old, new)


def make(name):
    s = open(SRC).read()
    if name == "noflush":
        s = sub(s, "if (last || nrow == kFlushRows) {", "if ((last || nrow == kFlushRows) && A.n_cols < 0) {")
    elif name == "nowin":
        s = sub(s, """        LDS v4u* w4 = reinterpret_cast<LDS v4u*>(win);
        w4[lane] = cc.w0;
        w4[64 + lane] = cc.w1;
        if (lane < 8) w4[128 + lane] = cc.w2;
      }
      RowC cn;""", """        LDS v4u* w4 = reinterpret_cast<LDS v4u*>(win);
        if (A.n_cols < 0) {
        w4[lane] = cc.w0;
        w4[64 + lane] = cc.w1;
        if (lane < 8) w4[128 + lane] = cc.w2;
        }
      }
      RowC cn;""")
    elif name == "noruns":
        s = sub(s, "            if (v != 0u) {\n              const int s = max(ck",
                "            if (v != 0u && A.n_cols < 0) {\n              const int s = max(ck")
    elif name == "rp_lds":
        os.makedirs(TMP, exist_ok=True)
        p = os.path.join(TMP, "rp_lds.hip")
        open(p, "w").write(s)
        subprocess.run(["patch", "-s", p, os.path.join(REPO, "profiles/variants/row_prefix_lds.patch")], check=True)
        s = open(p).read()
    elif name in ("rowlist8", "rowlist8mid"):  # the row-list patch at 8 waves per workgroup (2 per CU)
        os.makedirs(TMP, exist_ok=True)
        p = os.path.join(TMP, f"{name}.hip")
        open(p, "w").write(s)
        subprocess.run(["patch", "-s", p, os.path.join(REPO, "profiles/variants/tile_counts_rowlist16.patch")], check=True)
        s = open(p).read()
        s = sub(s, "constexpr int kCntWaves = 16;", "constexpr int kCntWaves = 8;")
        s = sub(s, "constexpr int kRowList = 8192;", "constexpr int kRowList = 2048;")  # (2 workgroups per CU)
        s = sub(s, "void tile_counts(const pw_msa_args A", "void tile_counts(const pw_msa_args A")
        s = s.replace("__global__ __launch_bounds__(64 * kCntWaves, 1) void tile_counts", "__global__ __launch_bounds__(64 * kCntWaves, 4) void tile_counts")
        if name == "rowlist8":
            s = sub(s, "  const int tile = tile_of_block((int)blockIdx.x, (int)gridDim.x);", "  const int tile = (int)blockIdx.x;")
    elif name == "k1_3ahead":  # row_chunk_sums with three groups' loads in flight (unrolled by three)
        s = sub(s, """  SumPre p0, p1;
  sums_load(A, sums_desc(A, sdesc, g, lane), g, lane, p0);
  sums_load(A, sums_desc(A, sdesc, g + nw, lane), g + nw, lane, p1);
  uint64_t dn = sums_desc(A, sdesc, g + 2 * nw, lane);""", """  SumPre p0, p1, p2;
  sums_load(A, sums_desc(A, sdesc, g, lane), g, lane, p0);
  sums_load(A, sums_desc(A, sdesc, g + nw, lane), g + nw, lane, p1);
  sums_load(A, sums_desc(A, sdesc, g + 2 * nw, lane), g + 2 * nw, lane, p2);
  uint64_t dn = sums_desc(A, sdesc, g + 3 * nw, lane);""")
        s = sub(s, """    const uint64_t dnn = sums_desc(A, sdesc, g + 3 * nw, lane);
    asm volatile("" : "+v"(dn)::"memory");
    sums_load(A, dn, g + 2 * nw, lane, p);""", """    const uint64_t dnn = sums_desc(A, sdesc, g + 4 * nw, lane);
    asm volatile("" : "+v"(dn)::"memory");
    sums_load(A, dn, g + 3 * nw, lane, p);""")
        s = sub(s, """  for (uint32_t k = 2; k <= n_mine; k += 2) {
    step(p0);
    step(p1);
  }
  if (n_mine & 1) step(p0);""", """  for (uint32_t k = 3; k <= n_mine; k += 3) {
    step(p0);
    step(p1);
    step(p2);
  }
  if (n_mine % 3 >= 1) step(p0);
  if (n_mine % 3 == 2) step(p1);""")
    elif name == "k1_32b":  # profiles/variants/row_chunk_sums_32bases.patch
        os.makedirs(TMP, exist_ok=True)
        p = os.path.join(TMP, "k1_32b.hip")
        open(p, "w").write(s)
        subprocess.run(["patch", "-s", p, os.path.join(REPO, "profiles/variants/row_chunk_sums_32bases.patch")], check=True)
        s = open(p).read()
    elif name.startswith("k1g"):  # row_chunk_sums grid of N workgroups (product: 2048)
        n = int(name[3:])
        s = sub(s, "(nb1 < 2048 ? nb1 : 2048)", f"(nb1 < {n} ? nb1 : {n})")
    elif name.startswith("sy"):  # slot_rows with N workgroups per row (product: 2048 / rows, <= 64)
        s = sub(s, "const unsigned sy = a->n_rows >= 2048 ? 1u : (2048u / a->n_rows < 64u ? 2048u / a->n_rows : 64u);",
                f"const unsigned sy = {int(name[2:])}u;")
    elif name == "nogather":  # no window reads at all (the group bytes are a constant)
        s = sub(s, """            const uint32_t s4 = __builtin_amdgcn_alignbyte(p[1], p[0], (uint32_t)src & 3u);""",
                """            const uint32_t s4 = 0x41434754u + (uint32_t)(src & 0) + (uint32_t)(p == nullptr);""")
    elif name == "ofs_nt":  # row_chunk_sums' ofs loads non-temporal (once-read stream)
        s = sub(s, "  p.q0 = src[0];\n  p.q1 = src[1];", "  p.q0 = __builtin_nontemporal_load(src);\n  p.q1 = __builtin_nontemporal_load(src + 1);")
    elif name == "seq_nt":  # tile_counts' base-window loads non-temporal
        for k in ("o + 16u * (uint32_t)lane, 0, 0);", "o + 1024u + 16u * (uint32_t)lane, 0, 0);",
                  "o + 2048u + 16u * (uint32_t)(lane & 7), 0, 0);"):
            s = sub(s, k, k.replace(", 0, 0);", ", 0, 2);"))
    elif name == "cnt_nt":  # tile_counts' counter table / consensus stores non-temporal
        s = sub(s, "    dst[i] = (int32_t)tab[f * kCntW + cnt_swz(c)];", "    __builtin_nontemporal_store((int32_t)tab[f * kCntW + cnt_swz(c)], dst + i);")
        s = sub(s, "      A.consensus[c0 + c] = best;\n      if (cons_star && c0 + c >= zlo && c0 + c <= zhi) cons_star[c0 + c - zlo] = best == '-' ? (uint8_t)'*' : best;",
                "      __builtin_nontemporal_store(best, A.consensus + c0 + c);\n      if (cons_star && c0 + c >= zlo && c0 + c <= zhi) __builtin_nontemporal_store(best == '-' ? (uint8_t)'*' : best, cons_star + c0 + c - zlo);")
    elif name == "winpad":  # tile_counts' base window padded one dword per eight (no 8-way read conflicts)
        s = sub(s, "  uint32_t win[kCntWaves][kWin / 4];", "  uint32_t win[kCntWaves][kWin / 4 + kWin / 32 + 8];")
        s = sub(s, "__device__ __forceinline__ uint32_t bin_codes5(", "typedef unsigned int v4a4 __attribute__((ext_vector_type(4), aligned(4)));\n__device__ __forceinline__ uint32_t bin_codes5(")
        s = sub(s, """        LDS v4u* w4 = reinterpret_cast<LDS v4u*>(win);
        w4[lane] = cc.w0;
        w4[64 + lane] = cc.w1;
        if (lane < 8) w4[128 + lane] = cc.w2;""", """        *reinterpret_cast<LDS v4a4*>(win + 4 * lane + (lane >> 1)) = cc.w0;
        *reinterpret_cast<LDS v4a4*>(win + 288 + 4 * lane + (lane >> 1)) = cc.w1;
        if (lane < 8) *reinterpret_cast<LDS v4a4*>(win + 576 + 4 * lane + (lane >> 1)) = cc.w2;""")
        s = sub(s, """          LDS v4u* w4 = reinterpret_cast<LDS v4u*>(win);
          w4[lane] = w0;
          w4[64 + lane] = w1;
          if (lane < 8) w4[128 + lane] = w2;""", """          *reinterpret_cast<LDS v4a4*>(win + 4 * lane + (lane >> 1)) = w0;
          *reinterpret_cast<LDS v4a4*>(win + 288 + 4 * lane + (lane >> 1)) = w1;
          if (lane < 8) *reinterpret_cast<LDS v4a4*>(win + 576 + 4 * lane + (lane >> 1)) = w2;""")
        s = sub(s, """            const LDS uint32_t* p = reinterpret_cast<const LDS uint32_t*>(wb + (src & ~3));
            const uint32_t s4 = __builtin_amdgcn_alignbyte(p[1], p[0], (uint32_t)src & 3u);""", """            const int dd = src >> 2, de = dd + 1;
            const uint32_t s4 = __builtin_amdgcn_alignbyte(win[de + (de >> 3)], win[dd + (dd >> 3)], (uint32_t)src & 3u);""")
    elif name == "k1_sumonly":  # timing only: row_chunk_sums loads and sums, no run entries / stores of runs
        s = sub(s, "  const int cs = sums_group(A, p, lane, (LDS uint16_t*)lr32);",
                "  int cs = 0;\n    { uint32_t t = p.q0.x + p.q0.y + p.q0.z + p.q0.w + p.q1.x + p.q1.y + p.q1.z + p.q1.w; cs = (int)row16_scan_incl(t); }")
    elif name == "head":
        s = subprocess.run(["git", "-C", REPO, "show", "HEAD:pwasm_amd/csrc/pw_msa.hip"], check=True,
                           capture_output=True, text=True).stdout
    elif name != "cur":
        raise SystemExit(f"unknown variant {name}")
    os.makedirs(TMP, exist_ok=True)
    p = os.path.join(TMP, f"{name}.hip")
    open(p, "w").write(s)
    return p


if __name__ == "__main__":
    names = sys.argv[1:] or ["cur", "noflush", "nowin", "noruns", "rp_lds"]
    args = [f"{n}={make(n)}" for n in names]
    subprocess.run([sys.executable, os.path.join(REPO, "tools/exp_msa.py"), *args], check=True)
