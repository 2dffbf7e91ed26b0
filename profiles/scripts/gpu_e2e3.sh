#!/bin/bash
# On the GPU box: where cfg3's end-to-end CLI time goes.  The full 10M-record cfg3 PAF, the CLI with
# PW_PROFILE_HOST=1 (per-batch phases), and the file system's own write rate for the same bytes
# (16 threads, pwrite of 64 MB blocks), so the CLI's output rate can be read against it.
# Usage: profiles/scripts/gpu_e2e3.sh <tag> [scale]
set -uo pipefail
TAG=${1:-e3}; S=${2:-1.0}
O=gpurun_out/e2e_$TAG
mkdir -p $O
export TMPDIR=/tmp
D=$(mktemp -d /tmp/pwe2e.XXXX)
df -h /tmp > $O/df.txt 2>&1; mount | grep -E " /tmp | / " >> $O/df.txt 2>&1; nproc >> $O/df.txt
timeout -k 10 300 synth/build/pwsynth paf --config 3 --scale $S --seed 3 --fa $D/q.fa --paf $D/a.paf --threads 16 2> $O/synth.err || { echo "synth failed"; exit 1; }
ls -la $D >> $O/df.txt
T0=$(date +%s.%N); timeout -k 10 300 env PW_PROFILE_HOST=1 pwasm_amd/bin/pafreport -G -C -r $D/q.fa $D/a.paf -o $D/r.txt 2> $O/cli.err || { echo "cli failed: $?"; tail -20 $O/cli.err; exit 1; }
T1=$(date +%s.%N); echo "cli wall $(python3 -c "print(round($T1 - $T0, 3))") s" >> $O/df.txt; ls -la $D/r.txt >> $O/df.txt
rm -f $D/r.txt
timeout -k 10 300 python3 - "$D" > $O/write_rate.txt 2>&1 <<'EOF' || { echo "write test failed"; exit 1; }
import os, sys, time, threading
d = sys.argv[1]
size = int(float(os.environ.get("PW_WBYTES", 16.4e9)))
blk = 64 << 20
buf = os.urandom(blk)
for nt in (1, 4, 16):
    p = os.path.join(d, f"w{nt}.bin")
    fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    os.ftruncate(fd, size)
    nb = size // blk
    t0 = time.perf_counter()
    def work(t):
        for k in range(t, nb, nt):
            os.pwrite(fd, buf, k * blk)
    th = [threading.Thread(target=work, args=(t,)) for t in range(nt)]
    [x.start() for x in th]
    [x.join() for x in th]
    el = time.perf_counter() - t0
    os.close(fd)
    print(f"{nt} threads: {nb * blk / el / 1e9:.2f} GB/s ({el:.2f} s for {nb * blk / 1e9:.1f} GB)", flush=True)
    os.remove(p)
EOF
cat $O/write_rate.txt
grep -E "^\[cli\]" $O/cli.err | tail -30; cat $O/df.txt
rm -rf $D
