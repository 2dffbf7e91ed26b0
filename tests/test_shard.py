"""Multi-GPU shard/merge path on the CPU: splitting a PAF by target, running each
shard on its own and merging the line-tagged item streams must reproduce a single-process run
byte for byte (stdout, stderr, exit code).  Shards are run by the oracle here (no GPU); the
world_size-2 case goes through torch.distributed with the gloo backend.  The HIP path of the
same merge is in test_gpu_parity.py::test_sharded_run_on_gpu."""
import os
import random
import socket

import pytest

from conftest import ORACLE, run, synth_paf
from pwasm_amd import shard


def _oracle_items(fa, shard_paf, items_path, flags=()):
    rc, out, err = run([ORACLE, "--items", items_path, *flags, "-r", fa, shard_paf])
    assert out == b"" and err == b"", (out[:200], err[:200])
    return shard.read_items(items_path)


def _check_split(fa, paf, tmp_path, world, flags=()):
    want = run([ORACLE, *flags, "-r", fa, paf])
    parts = shard.split_paf(paf, world, str(tmp_path), prefix=f"w{world}_")
    got_items = []
    for r, (p, gmap) in enumerate(parts):
        got_items.append((_oracle_items(fa, p, str(tmp_path / f"w{world}_{r}.pwi"), flags), gmap))
    out, err, rc = shard.merge_items(got_items)
    assert (rc, out, err) == want
    return parts


def _with_duplicates_and_comments(paf, tmp_path, seed):
    """Repeat some records (gene-mode q~t dedupe warnings) and add comment lines."""
    lines = open(paf).read().splitlines(keepends=True)
    rng = random.Random(seed)
    out = ["# header comment\n"]
    for ln in lines:
        out.append(ln)
        if rng.random() < 0.05:
            out.append(ln)
        if rng.random() < 0.02:
            out.append("# comment\n")
    p = tmp_path / "dup.paf"
    p.write_text("".join(out))
    return str(p)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_split_merge_equals_single_run(built, tmp_path, world):
    fa, paf = synth_paf(tmp_path, 0, seed=5)
    parts = _check_split(fa, paf, tmp_path, world)
    n = sum(len(g) for _, g in parts)
    assert n == len([l for l in shard.read_lines(paf) if not l.startswith(b"#")])
    assert sum(1 for _, g in parts if g) > 1  # the split is not degenerate


def test_split_keeps_dedupe_and_comments(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 0, seed=6)
    dup = _with_duplicates_and_comments(paf, tmp_path, 1)
    _, _, err = run([ORACLE, "-r", fa, dup])
    assert b"already seen" in err
    _check_split(fa, dup, tmp_path, 4)


@pytest.mark.parametrize("kind", ["mismatch", "bounds"])
def test_split_stops_at_first_fatal(built, tmp_path, kind):
    from test_gpu_parity import _inject
    fa, paf = synth_paf(tmp_path, 0, seed=41)
    bad = _inject(paf, tmp_path, kind, seed=5)
    rc, _, _ = run([ORACLE, "-r", fa, bad])
    assert rc == 1
    _check_split(fa, bad, tmp_path, 3)


def test_split_modes(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 0, seed=12)
    for flags in (["-F"], ["-N"], ["-G", "-C"]):
        _check_split(fa, paf, tmp_path, 2, flags)


def test_line_reader_matches_glinereader(tmp_path):
    p = tmp_path / "x.paf"
    p.write_bytes(b"a\r\nb\rc\n\nd")
    assert shard.read_lines(str(p)) == [b"a", b"b", b"c", b"", b"d"]
    p.write_bytes(b"a\n")
    assert shard.read_lines(str(p)) == [b"a"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_rank(rank, world, port, fa, paf, tmp, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # every rank computes the same split; each runs only its own shard
        parts = shard.split_paf(paf, world, tmp, prefix=f"g{rank}_")
        p, gmap = parts[rank]
        items = _oracle_items(fa, p, os.path.join(tmp, f"g{rank}.pwi"))
        gathered = [None] * world
        dist.all_gather_object(gathered, (items, gmap))
        if rank == 0:
            q.put(shard.merge_items(gathered))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_world_size_2(built, tmp_path):
    import torch.multiprocessing as mp
    fa, paf = synth_paf(tmp_path, 0, seed=7)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_rank, args=(r, 2, port, fa, paf, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    out, err, rc = res
    assert (rc, out, err) == run([ORACLE, "-r", fa, paf])
