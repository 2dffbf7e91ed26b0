"""Per-kernel resource usage of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage), one
line per kernel: VGPRs, AGPRs, SGPRs, spills, occupancy, LDS.
Usage: python tools/kres.py pwasm_amd/csrc/pw_report.hip [extra hipcc flags]"""
import re
import subprocess
import sys

REPO = __file__.rsplit("/tools/", 1)[0]


def main(src, extra):
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", f"-I{REPO}/include", f"-I{REPO}/pwasm_amd/csrc"]
    if src.endswith("pw_report.hip") and not extra:
        extra = ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]
    p = subprocess.run(["/opt/rocm/bin/hipcc", *flags, *extra, "-c", src, "-o", "/tmp/kres.o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    cur, rows = None, []
    for ln in p.stderr.splitlines():
        m = re.search(r"remark: \s*(.+?) \[-Rpass-analysis", ln)
        if not m:
            continue
        k, _, v = m.group(1).partition(": ")
        if k == "Function Name":
            cur = {"name": re.sub(r"^_ZN2pw\d+", "", v).split("E", 1)[0]}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for r in rows:
        print(f"{r['name'][:24]:24s} vgpr {r.get('VGPRs', '?'):>4s} agpr {r.get('AGPRs', '?'):>3s} "
              f"sgpr {r.get('TotalSGPRs', '?'):>4s} spill s{r.get('SGPRs Spill', '?')}/v{r.get('VGPRs Spill', '?')} "
              f"occ {r.get('Occupancy [waves/SIMD]', '?'):>2s} lds {r.get('LDS Size [bytes/block]', '?')}")
    if p.returncode:
        print(p.stderr[-3000:])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
