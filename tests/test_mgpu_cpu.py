"""CPU: the pieces of the multi-GPU pafreport driver (pwasm_amd/mgpu.py) that need no GPU — the
ragged all-gather of per-genome rows / names over gloo (world 2), the C++ k-way merge of the
shards' item streams (pw_items_merge) against the Python reference merge (shard.merge_items),
GArgs-style option parsing and the genome-table writer."""
import os
import socket
import struct

import numpy as np
import pytest
import torch.multiprocessing as mp

import pwasm_amd as pw
from pwasm_amd import mgpu, shard


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = torch.arange(3 + 4 * rank, dtype=torch.int64) + 100 * rank
        got = mgpu.gather_ragged(t)
        q.put((rank, [x.tolist() for x in got]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gather_ragged_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_gather_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [list(range(3)), [100 + k for k in range(7)]]
    assert res[0] == want and res[1] == want


def _write_items(path, items):
    with open(path, "wb") as f:
        f.write(b"PWI1")
        for line, st, o, e in items:
            f.write(struct.pack("<QiII", line, st, len(o), len(e)) + o + e)


@pytest.mark.parametrize("stop", [None, 7])
def test_items_merge_matches_python_merge(built, tmp_path, stop):
    rng = np.random.default_rng(3)
    lines = rng.permutation(40)
    shards = [sorted(lines[k::3].tolist()) for k in range(3)]
    paths, parts = [], []
    for k, ls in enumerate(shards):
        items = [(ln, 1 if ln == stop else -1, f"out{ln}\n".encode() * (ln % 3), f"err{ln}\n".encode() * (ln % 2))
                 for ln in ls]
        p = tmp_path / f"s{k}.pwi"
        _write_items(p, items)
        paths.append(p)
        parts.append((shard.read_items(str(p)), list(range(100))))  # identity line map
    want_out, want_err, want_rc = shard.merge_items(parts)
    rc = pw.items_merge(paths, tmp_path / "o.txt", tmp_path / "e.txt")
    assert rc == want_rc
    assert (tmp_path / "o.txt").read_bytes() == want_out
    assert (tmp_path / "e.txt").read_bytes() == want_err


def test_parse_args():
    o, n, x = mgpu.parse_args(["-G", "-C", "-rq.fa", "a.paf", "-o", "r.txt", "--genome-table", "t.tsv"])
    assert o == {"G": "", "C": "", "r": "q.fa", "o": "r.txt"} and n == ["a.paf"] and x == {"genome-table": "t.tsv"}
    o, n, _ = mgpu.parse_args(["-GC", "-r", "q.fa", "a.paf"])
    assert o == {"G": "", "C": "", "r": "q.fa"}
    with pytest.raises(SystemExit):
        mgpu.parse_args(["-x"])


def test_genome_table_writer(tmp_path):
    rows = np.zeros(32, np.uint8)
    rows[0:4] = np.frombuffer(np.uint32(3).tobytes(), np.uint8)
    rows[4:8] = np.frombuffer(np.uint32(17).tobytes(), np.uint8)
    rows[8:16] = np.frombuffer(np.uint64(12345).tobytes(), np.uint8)
    rows[16:20] = np.frombuffer(np.uint32(1).tobytes(), np.uint8)
    p = tmp_path / "t.tsv"
    mgpu.write_genome_table(p, [rows], [[b"tA", b"tB"]])
    assert p.read_text().splitlines()[1:] == ["tA\t3\t17\t12345", "tB\t1\t0\t0"]
