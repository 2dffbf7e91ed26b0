import sys, pathlib; sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent.parent))
import bench, pwasm_amd as pw, subprocess, tempfile, os
t = tempfile.mkdtemp(); fa = os.path.join(t, "q.fa"); paf = os.path.join(t, "a.paf")
subprocess.run(["synth/build/pwsynth", "paf", "--config", "2", "--seed", "2", "--fa", fa, "--paf", paf], check=True, stderr=subprocess.DEVNULL)
print(bench.gpu_pack_check(pw, paf))
