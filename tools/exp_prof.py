"""Experiment (GPU box): region timings of the `prof` build's render_kernel (s_memtime probes,
tools/exp_build.py) on cfg2.  Usage: PWASM_LIB=tools/abl_build/prof/lib/libpwasm_amd.so python3 tools/exp_prof.py"""
import ctypes
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import pwasm_amd as pw  # noqa: E402

NAMES = ["setup+wait (pre_ready, qw)", "head: type/rloc/aa", "bases + tloc", "tctx", "qctx + status", "codon impact",
         "modseq err, next Hot decode", "next chunk loads issue", "line scan, page, results", "ostart/cmap",
         "gather + loop tail", "rloc + aa codon", "indel codons", "sub impact (then-branch)", "-", "-"]


def main():
    tmp = tempfile.mkdtemp()
    fa, paf = os.path.join(tmp, "q.fa"), os.path.join(tmp, "a.paf")
    subprocess.run([os.path.join(REPO, "synth/build/pwsynth"), "paf", "--config", "2", "--seed", "2", "--fa", fa,
                    "--paf", paf], check=True, stderr=subprocess.DEVNULL)
    batch = pw.HostBatch(fa, paf, pw.FLAG_G | pw.FLAG_C)
    dev = pw.stage_batch(batch, "cuda:0")
    sp = torch.cuda.current_stream().cuda_stream
    L = pw.lib()
    L.pw_exp_prof.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 16)()
    for _ in range(3):
        pw.run_report(batch, dev, sp)
    torch.cuda.synchronize()
    L.pw_exp_prof(buf)
    n = 5
    for _ in range(n):
        pw.run_report(batch, dev, sp)
    torch.cuda.synchronize()
    assert L.pw_exp_prof(buf) == 0
    v = [buf[i] / n for i in range(16)]
    tot = sum(v)
    for i, name in enumerate(NAMES[:16]):
        print(f"{i:2d} {name:32s} {v[i] / 1e6:10.2f} Mclk/pass  {100 * v[i] / tot:5.1f} %")
    print(f"   total {tot / 1e6:.2f} Mclk/pass (summed over waves)")


if __name__ == "__main__":
    main()
