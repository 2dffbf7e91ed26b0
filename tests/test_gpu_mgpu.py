"""GPU: the multi-GPU pafreport driver (pwasm_amd/mgpu.py) with 2 and 3 ranks, each packing its
target-genome shard and running the HIP pass (all ranks on cuda:0 here, collectives over gloo —
RCCL refuses two ranks on one GPU; on a node every rank has its own GPU and the backend is
"nccl").  The merged report, stderr and exit code must equal the single-process oracle run; the
node-wide per-genome table must equal one computed from the PAF and the oracle's report."""
import collections
import os
import queue
import socket
import time

import pytest
import torch.multiprocessing as mp

from conftest import ORACLE, run, synth_paf
from test_gpu_parity import _inject
from test_shard import _with_duplicates_and_comments

pytestmark = pytest.mark.gpu


def _rank(rank, world, port, argv, errf, q, backend="gloo", env=None):
    import faulthandler
    tb = open(f"{errf}.rank{rank}.tb", "w")
    faulthandler.dump_traceback_later(100, exit=True, file=tb)  # a hung rank names where it hangs
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PW_DIST_BACKEND=backend, **(env or {}))
    if rank == 0:
        fd = os.open(errf, os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
        os.dup2(fd, 2)
        if os.environ.get("PW_TEST_STDOUT"):  # (rank 0's stdout into a file)
            fo = os.open(os.environ["PW_TEST_STDOUT"], os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
            os.dup2(fo, 1)
    from pwasm_amd import mgpu
    import torch.distributed as dist
    rc = mgpu.main(argv)
    if dist.is_initialized():
        dist.destroy_process_group()
    q.put((rank, rc))


def run_mgpu(world, argv, tmp_path, backend="gloo", env=None):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    errf = str(tmp_path / "mg.err")
    ps = [ctx.Process(target=_rank, args=(r, world, port, argv, errf, q, backend, env)) for r in range(world)]
    for p in ps:
        p.start()
    rcs = {}
    deadline = time.time() + 150
    while len(rcs) < world:  # (fail as soon as a rank dies or hangs, with its traceback)
        try:
            r, rc = q.get(timeout=5)
            rcs[r] = rc
            continue
        except queue.Empty:
            pass
        dead = [p.exitcode for p in ps if p.exitcode not in (None, 0)]
        if dead or time.time() > deadline:
            for p in ps:
                p.kill()
            tbs = "".join(open(f"{errf}.rank{r}.tb").read() for r in range(world) if os.path.exists(f"{errf}.rank{r}.tb"))
            raise AssertionError(f"ranks exit {dead or 'hung'}; stderr: {open(errf, 'rb').read()[-2000:]!r}\n{tbs}")
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(set(rcs.values())) == 1
    # rank 0's stderr also carries runtime noise from before the driver starts (libdrm, c10d)
    noise = (b"/opt/amdgpu/", b"[W", b"[Gloo]", b"[I")
    err = b"".join(ln for ln in open(errf, "rb").read().splitlines(keepends=True) if not ln.startswith(noise))
    return rcs[0], err


def _genome_table_from(paf, report):
    recs = [ln.split("\t") for ln in open(paf).read().splitlines() if ln and not ln.startswith("#")]
    blocks = report.decode().split(">")[1:]
    tab = collections.OrderedDict()
    # records in report order are the PAF's kept records (dedupe / self alignments removed):
    # match them by their header's target label
    it = iter(recs)
    for blk in blocks:
        hdr = blk.split("\n", 1)[0]
        tl = hdr.split(" ")[0].split("--")[-1]
        while True:
            f = next(it)
            if f"{f[5]}:{f[7]}-{f[8]}{f[4]}" == tl:
                break
        r = tab.setdefault(f[5], [0, 0, 0])
        r[0] += 1
        r[1] += blk.count("\n") - 1
        r[2] += int(f[8]) - int(f[7])
    return tab


@pytest.mark.parametrize("world,runner", [(2, "1"), (3, "1"), (2, "0")])
def test_mgpu_matches_single_process(built, tmp_path, world, runner):
    """runner "1": batches through pw_runner (GPU cs packing, the CLI's device session; the genome
    rows from its device results); "0": staged through torch tensors with host packing."""
    fa, paf = synth_paf(tmp_path, 0, seed=17)
    dup = _with_duplicates_and_comments(paf, tmp_path, 2)
    out = tmp_path / "r.txt"
    tab = tmp_path / "g.tsv"
    rc, err = run_mgpu(world, ["-r", fa, dup, "-o", str(out), "--genome-table", str(tab)], tmp_path,
                       env={"PW_MGPU_RUNNER": runner})
    orc, oout, oerr = run([ORACLE, "-r", fa, dup])
    assert (rc, out.read_bytes(), err) == (orc, oout, oerr)
    want = _genome_table_from(dup, oout)
    got = {}
    for ln in tab.read_text().splitlines()[1:]:
        t, a, e, b = ln.split("\t")
        got[t] = [int(a), int(e), int(b)]
    assert got == dict(want)


@pytest.mark.parametrize("kind", ["mismatch", "mismatch_splice", "bounds"])
def test_mgpu_fatal_midway(built, tmp_path, kind):
    """A fatal line two thirds in: a base mismatch, an unknown op byte after a flipped base (the GPU
    packer hands the record back to the host packer for the reference's error), a bounds violation."""
    fa, paf = synth_paf(tmp_path, 0, seed=41)
    bad = _inject(paf, tmp_path, kind, seed=5)
    out = tmp_path / "r.txt"
    rc, err = run_mgpu(2, ["-r", fa, bad, "-o", str(out)], tmp_path)
    orc, oout, oerr = run([ORACLE, "-r", fa, bad])
    assert (rc, out.read_bytes(), err) == (orc, oout, oerr) and orc == 1


@pytest.mark.parametrize("flags", [["-F"], ["-N"], ["-G"], ["-F", "-C"]])
def test_mgpu_modes(built, tmp_path, flags):
    """The report modes through the multi-GPU driver's runner path (GPU cs packing in every mode):
    full-genome, no codon analysis, gene mode, full-genome with codons forced."""
    fa, paf = synth_paf(tmp_path, 0, seed=23)
    dup = _with_duplicates_and_comments(paf, tmp_path, 2)
    out = tmp_path / "r.txt"
    rc, err = run_mgpu(2, [*flags, "-r", fa, dup, "-o", str(out)], tmp_path)
    orc, oout, oerr = run([ORACLE, *flags, "-r", fa, dup])
    assert (rc, out.read_bytes(), err) == (orc, oout, oerr)


def test_mgpu_cfg3_shards_gene_mode(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 3, scale=0.002)
    out = tmp_path / "r.txt"
    rc, err = run_mgpu(2, ["-G", "-C", "-r", fa, paf, "-o", str(out)], tmp_path)
    orc, oout, oerr = run([ORACLE, "-G", "-C", "-r", fa, paf])
    assert (rc, out.read_bytes(), err) == (orc, oout, oerr) and orc == 0


@pytest.mark.parametrize("window", [None, "37"])
def test_mgpu_many_batches_per_rank(built, tmp_path, window):
    """Each rank's lines in several pipelined batches (PW_CHUNK_BYTES): the q~t dedupe state moves
    from batch to batch, the output offsets span all of them; with PW_WINDOW_LINES the report is
    written in many windows of global lines while later batches are still being packed."""
    fa, paf = synth_paf(tmp_path, 0, seed=19)
    dup = _with_duplicates_and_comments(paf, tmp_path, 4)
    out = tmp_path / "r.txt"
    env = {"PW_CHUNK_BYTES": "4000", **({"PW_WINDOW_LINES": window} if window else {})}
    rc, err = run_mgpu(2, ["-r", fa, dup, "-o", str(out)], tmp_path, env=env)
    orc, oout, oerr = run([ORACLE, "-r", fa, dup])
    assert (rc, out.read_bytes(), err) == (orc, oout, oerr)


def test_mgpu_stdout_windows_fatal(built, tmp_path):
    """No -o, small windows, a fatal line two thirds in: rank 0 streams each window to stdout."""
    fa, paf = synth_paf(tmp_path, 0, seed=41)
    bad = _inject(paf, tmp_path, "mismatch", seed=5)
    so = tmp_path / "stdout.txt"
    rc, err = run_mgpu(3, ["-r", fa, bad], tmp_path,
                       env={"PW_TEST_STDOUT": str(so), "PW_CHUNK_BYTES": "20000", "PW_WINDOW_LINES": "50"})
    orc, oout, oerr = run([ORACLE, "-r", fa, bad])
    assert (rc, err) == (orc, oerr) and orc == 1
    assert so.read_bytes() == oout


def test_mgpu_stdout(built, tmp_path):
    """No -o: the file assembled at offsets goes to rank 0's stdout."""
    fa, paf = synth_paf(tmp_path, 0, seed=23)
    so = tmp_path / "stdout.txt"
    rc, err = run_mgpu(2, ["-r", fa, paf], tmp_path, env={"PW_TEST_STDOUT": str(so)})
    orc, oout, oerr = run([ORACLE, "-r", fa, paf])
    # (c10d's "[Gloo] Rank 0 is connected ..." goes to stderr: mgpu.main keeps it off stdout)
    got = so.read_bytes()
    assert (rc, err) == (orc, oerr)
    assert got == oout, f"stdout differs: {len(got)} vs {len(oout)} bytes, first at {_first_diff(got, oout)}"


def _first_diff(a, b):
    n = min(len(a), len(b))
    return next((i for i in range(n) if a[i] != b[i]), n)


@pytest.mark.skipif(__import__("torch").cuda.device_count() < 2, reason="needs two GPUs (RCCL ranks)")
def test_mgpu_rccl_two_gpus(built, tmp_path):
    """The node configuration: one rank per GPU, collectives over RCCL ("nccl")."""
    fa, paf = synth_paf(tmp_path, 0, seed=29)
    dup = _with_duplicates_and_comments(paf, tmp_path, 5)
    out = tmp_path / "r.txt"
    rc, err = run_mgpu(2, ["-r", fa, dup, "-o", str(out)], tmp_path, backend="nccl")
    orc, oout, oerr = run([ORACLE, "-r", fa, dup])
    assert (rc, out.read_bytes(), err) == (orc, oout, oerr)
