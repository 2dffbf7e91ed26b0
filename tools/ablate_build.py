"""Experiment builds (never shipped): copies of pw_report.hip with one part of the report line
switched off, linked into tools/abl_build/<name>/{lib,bin} so tools/ablate_run.sh can measure
what each part of render_kernel costs (SQ counters, duration).  Outputs differ from the product."""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "pwasm_amd/csrc/pw_report.hip")
OUT = os.path.join(REPO, "tools/abl_build")
PATCHES = {
    "base": [],
    "nocodon": [("  if (!skip) {\n    if (typ == PW_OP_SUB) {", "  if (false) {\n    if (typ == PW_OP_SUB) {")],
    "notctx": [("      if (in.tmode == 0) {\n        emit_tctx_fast(", "      if (false) {\n        emit_tctx_fast("),
               ("        o.put_span(in.tx, (int)(in.tx[0] & 0xFFu));\n", "")],
    "noqctx": [("      o.put_bytes(rv, 10);\n      o.put_bytes(sv, sl);\n", "")],
    "nohead": [("      wr_num(o, r.tab, (uint32_t)(e.rloc + 1));\n", ""), ("      wr_num(o, r.tab, (uint32_t)(aap0 + 1));\n", "")],
    "nocod_sub": [("    if (typ == PW_OP_SUB) {\n      const int p0 = e.rloc - e.r_trloc;", "    if (false) {\n      const int p0 = e.rloc - e.r_trloc;")],
    "nocod_indel": [("      indel_impact(k, r, e, in.ns_pre);\n", "")],
    "nocod_slow": [("    if (!indel_codons_fast(r, e, a, x, dl, mm, rr)) {", "    if (!indel_codons_fast(r, e, a, x, dl, mm, rr) && false) {")],
    "nocod_long": [("  } else {  // long insertion: the reference loop as is", "  } else if (false) {  // long insertion: the reference loop as is")],
    "nogather": [("for (uint32_t cc = (uint32_t)lane * 16; cc < B; cc += kWave * 16) {",
                  "for (uint32_t cc = (uint32_t)lane * 16; cc < 0u; cc += kWave * 16) {")],
}


def main(names):
    src = open(SRC).read()
    objs = [os.path.join(REPO, "pwasm_amd/build", f) for f in os.listdir(os.path.join(REPO, "pwasm_amd/build"))
            if f.endswith(".o") and f != "pw_report.o"]
    for name in names:
        s = src
        for a, b in PATCHES[name]:
            assert a in s, (name, a)
            s = s.replace(a, b)
        d = os.path.join(OUT, name)
        os.makedirs(os.path.join(d, "lib"), exist_ok=True)
        os.makedirs(os.path.join(d, "bin"), exist_ok=True)
        hip = os.path.join(d, "pw_report.hip")
        open(hip, "w").write(s)
        inc = ["-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "pwasm_amd/csrc")]
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", *inc, "-c", hip,
                        "-o", os.path.join(d, "pw_report.o")], check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                        os.path.join(d, "lib/libpwasm_amd.so"), os.path.join(d, "pw_report.o"), *objs, "-ldl"],
                       check=True)
        shutil.copy(os.path.join(REPO, "pwasm_amd/bin/pafreport"), os.path.join(d, "bin/pafreport"))
        os.remove(hip)
        os.remove(os.path.join(d, "pw_report.o"))
        print("built", name)


if __name__ == "__main__":
    main(sys.argv[1:] or list(PATCHES))
