"""Multi-GPU sharding of a pafreport run.

Records are independent (printDiffInfo depends only on the record and its query,
pafreport.cpp:885), except gene mode's first-occurrence `q~t` dedupe (pafreport.cpp:319-334),
which is keyed by (query, target).  So the PAF is split BY TARGET NAME (column 6): every
rank packs and runs its own shard with no data-path collective, writes its output as a PWI1
item stream (pw_batch_write_items: each item = what one input line printed, tagged with its
line number), and rank 0 merges the items by global line number up to the first fatal item.
The merged stdout/stderr/exit code equal a single-process run on the whole input.
"""
from __future__ import annotations

import os
import re
import struct
import zlib

_EOL = re.compile(rb"\r\n|\r|\n")


def read_lines(path: str) -> list[bytes]:
    """Lines as GLineReader::getLine sees them (\\n, \\r or \\r\\n; no empty last line)."""
    data = open(path, "rb").read()
    lines = _EOL.split(data)
    if lines and lines[-1] == b"":
        lines.pop()
    return lines


def shard_of(line: bytes, world: int) -> int:
    """Rank of one PAF line: crc32 of the target name (PAF column 6).  Lines too short to have
    one are fatal wherever they land (pafreport.cpp:307-309) and go to rank 0."""
    f = line.split(b"\t", 6)
    if len(f) < 7:
        return 0
    return zlib.crc32(f[5]) % world


def split_paf(paf: str, world: int, out_dir: str, prefix: str = "shard") -> list[tuple[str, list[int]]]:
    """Write `world` shard files; returns [(path, global line number of each shard line)].
    Comment lines print nothing and are dropped."""
    lines = read_lines(paf)
    parts: list[list[bytes]] = [[] for _ in range(world)]
    gidx: list[list[int]] = [[] for _ in range(world)]
    for i, ln in enumerate(lines):
        if ln[:1] == b"#":
            continue
        r = shard_of(ln, world)
        parts[r].append(ln)
        gidx[r].append(i)
    out = []
    for r in range(world):
        p = os.path.join(out_dir, f"{prefix}{r}.paf")
        with open(p, "wb") as f:
            for ln in parts[r]:
                f.write(ln + b"\n")
        out.append((p, gidx[r]))
    return out


def read_items(path: str) -> list[tuple[int, int, bytes, bytes]]:
    """PWI1 stream -> [(local line, status, stdout bytes, stderr bytes)]."""
    data = open(path, "rb").read()
    if data[:4] != b"PWI1":
        raise ValueError(f"{path}: not a PWI1 item stream")
    pos, items = 4, []
    while pos < len(data):
        line, st, no, ne = struct.unpack_from("<QiII", data, pos)
        pos += 20
        o = data[pos:pos + no]
        pos += no
        e = data[pos:pos + ne]
        pos += ne
        items.append((line, st, o, e))
    return items


def merge_items(shards: list[tuple[list[tuple[int, int, bytes, bytes]], list[int]]]) -> tuple[bytes, bytes, int]:
    """Merge per-shard items [(items, global line map)] -> (stdout, stderr, exit code)."""
    allit = []
    for items, gmap in shards:
        for line, st, o, e in items:
            allit.append((gmap[line], st, o, e))
    allit.sort(key=lambda x: x[0])
    out, err = [], []
    for _, st, o, e in allit:
        out.append(o)
        err.append(e)
        if st >= 0:
            return b"".join(out), b"".join(err), st
    return b"".join(out), b"".join(err), 0
