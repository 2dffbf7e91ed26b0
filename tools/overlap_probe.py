"""Would two report passes on two HIP streams overlap into less than twice one pass?  (Host tool:
the cfg2 batch staged twice, K passes of each copy either back to back on one stream or interleaved
on two streams, HIP events around each form.)  Usage: python tools/overlap_probe.py [K]"""
import os
import subprocess
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pwasm_amd as pw  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
t = tempfile.mkdtemp()
fa, paf = os.path.join(t, "q.fa"), os.path.join(t, "a.paf")
subprocess.run([os.path.join(pw.REPO, "synth/build/pwsynth"), "paf", "--config", "2", "--seed", "2", "--fa", fa, "--paf",
                paf], check=True, stderr=subprocess.DEVNULL)
b = pw.HostBatch(fa, paf, pw.FLAG_G | pw.FLAG_C)
devs = [pw.stage_batch(b, "cuda:0") for _ in range(2)]
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
for d, s in zip(devs, (s0, s1)):
    pw.run_report(b, d, s.cuda_stream)
torch.cuda.synchronize()


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    fn()
    for s in (s0, s1):
        torch.cuda.current_stream().wait_stream(s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def serial():
    s0.wait_stream(torch.cuda.current_stream())
    for _ in range(K):
        pw.run_report(b, devs[0], s0.cuda_stream)
        pw.run_report(b, devs[1], s0.cuda_stream)


def overlapped():
    for s in (s0, s1):
        s.wait_stream(torch.cuda.current_stream())
    for _ in range(K):
        pw.run_report(b, devs[0], s0.cuda_stream)
        pw.run_report(b, devs[1], s1.cuda_stream)


for rep in range(3):
    a = timed(serial)
    c = timed(overlapped)
    print(f"rep {rep}: {2 * K} passes, one stream {a / (2 * K):.4f} ms/pass, two streams {c / (2 * K):.4f} ms/pass "
          f"({c / a:.3f}x)", flush=True)
