"""The GPU cs packer alone (bench.gpu_pack_check: cfg2's 100k cs strings, parity against the host
packer, HIP-event timing) — for kernel traces / PMC passes of pack_cs_kernel.
Usage: python tools/pack_bench.py [reps]"""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import pwasm_amd as pw  # noqa: E402

if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    with tempfile.TemporaryDirectory() as tmp:
        fa, paf = os.path.join(tmp, "q.fa"), os.path.join(tmp, "a.paf")
        subprocess.run([os.path.join(REPO, "synth/build/pwsynth"), "paf", "--config", "2", "--scale", "1.0", "--seed", "2",
                        "--fa", fa, "--paf", paf], check=True, stderr=subprocess.DEVNULL)
        print(json.dumps(bench.gpu_pack_check(pw, paf, reps=reps)))
