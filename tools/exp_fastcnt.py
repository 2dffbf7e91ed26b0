"""Experiment (GPU box): how many render_kernel waves take the fast emit_event instantiation on
cfg2.  Usage: PWASM_LIB=tools/abl_build/fastcnt/lib/libpwasm_amd.so python3 tools/exp_fastcnt.py"""
import ctypes
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import pwasm_amd as pw  # noqa: E402


def main():
    tmp = tempfile.mkdtemp()
    fa, paf = os.path.join(tmp, "q.fa"), os.path.join(tmp, "a.paf")
    subprocess.run([os.path.join(REPO, "synth/build/pwsynth"), "paf", "--config", "2", "--seed", "2", "--fa", fa,
                    "--paf", paf], check=True, stderr=subprocess.DEVNULL)
    batch = pw.HostBatch(fa, paf, pw.FLAG_G | pw.FLAG_C)
    dev = pw.stage_batch(batch, "cuda:0")
    L = pw.lib()
    L.pw_exp_prof.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 16)()
    pw.run_report(batch, dev, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert L.pw_exp_prof(buf) == 0
    fw, sw, nf, na = buf[0], buf[1], buf[2], buf[3]
    print(f"fast waves {fw}, general waves {sw} ({sw / max(fw + sw, 1):.3f}), lanes not fast {nf} of {na} "
          f"({nf / max(na, 1):.4f})")


if __name__ == "__main__":
    main()
