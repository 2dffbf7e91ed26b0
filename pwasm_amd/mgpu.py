"""Multi-GPU `pafreport`: one process per GPU, launched by torchrun.

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m pwasm_amd.mgpu [-G|-F] [-C|-N] -r cds.fa mappings.paf [-o report.txt] [--genome-table t.tsv]

Replaces the reference's sequential record loop (pafreport.cpp:303-436) over a node:

  read + route  rank r reads only bytes [r*S/N, (r+1)*S/N) of the PAF (pw_paf_split: the lines
                starting there, cut as the CLI cuts them) and sends each line to the rank owning
                its target genome (crc32 of PAF column 6 mod world) with its global input line
                (exclusive scan of the ranges' line counts): two all_to_all_single calls (RCCL over
                xGMI with the nccl backend).  Gene mode's first-occurrence q~t dedupe
                (pafreport.cpp:319-334) is keyed by the target, so it stays shard-local.
  batches       the rank's lines in pipelined batches (PW_CHUNK_BYTES, default 256 MB): batch k+1
                is packed on host threads while the GPU runs batch k (pw_batch_from_buffer, the
                dedupe state moving from batch to batch; pw_stop_table_build + pw_report_events).
  output        no rank-0 merge, written window by window of global input lines (OffsetWriter,
                PW_WINDOW_LINES) as the batches finish.  A rank holds the batches with lines in
                the current window or a later one (a batch stays pending until its last line's
                window is written), and waits in each window's collectives for the slowest rank.
                The first fatal input line of the window over all ranks ends the run
                (all-reduce MIN); every rank's per-line stdout byte counts of the window are summed
                over the ranks (all-reduce of one int64 per line of the window) and exclusive-scanned
                into file offsets after the previous windows, and each rank pwrites its own items
                there (pw_batch_write_range).  stderr lines (warnings, the fatal message) are
                gathered to rank 0 only and written in input-line order; the exit code is the fatal
                item's.  stdout without -o: the file is assembled in a temporary file and streamed
                out by rank 0 after each window.  c10d's connection messages are kept off stdout.
  per-genome    pw_genome_table sums each target's alignments / event lines / aligned bases on the
  tables        device; the rows and target names of all ranks are all-gathered (--genome-table).
No collective touches the per-record data path: records are independent.

PW_DIST_BACKEND=gloo runs the collectives on the host (tests put several ranks on one GPU,
which RCCL does not allow)."""
from __future__ import annotations

import ctypes
import os
import sys
import tempfile

import numpy as np

USAGE_OPTS = "DGFCNvd:p:r:o:m:w:c:s:"


def parse_args(argv):
    """GArgs-style option parsing (pafreport.cpp:177) + the driver's long options."""
    opts, nonopt, extra = {}, [], {}
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ("--genome-table", "--tmpdir"):
            extra[a[2:]] = argv[i + 1]
            i += 2
            continue
        if a.startswith("-") and len(a) > 1:
            k = 1
            while k < len(a):
                c = a[k]
                j = USAGE_OPTS.find(c)
                if j < 0 or c == ":":
                    raise SystemExit(f"Invalid argument: {a}")
                if j + 1 < len(USAGE_OPTS) and USAGE_OPTS[j + 1] == ":":
                    if k + 1 < len(a):
                        opts[c] = a[k + 1:]
                    else:
                        i += 1
                        opts[c] = argv[i]
                    break
                opts[c] = ""
                k += 1
        else:
            nonopt.append(a)
        i += 1
    return opts, nonopt, extra


def _gather(t, group=None):
    """all_gather of equally-shaped tensors (device tensors through the host under gloo)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    host = t.is_cuda and dist.get_backend(group) == "gloo"
    src = t.cpu() if host else t
    out = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(out, src, group=group)
    return out


def gather_ragged(t, group=None):
    """all_gather of 1-D tensors of different lengths: lengths first, then padded payloads."""
    import torch
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    lens = [int(x.item()) for x in _gather(n, group)]
    pad = torch.zeros(max(max(lens), 1), dtype=t.dtype, device=t.device)
    pad[: t.numel()] = t
    return [p[:k] for p, k in zip(_gather(pad, group), lens)]


def genome_rows(batch, dev, stream_ptr):
    """Per-genome rows of this rank's batch on the device (pw_genome_table) + target names."""
    import torch
    import pwasm_amd as pw
    gof, taln, names = batch.genomes()
    n = int(batch.view.n_alns)
    ng = len(names)
    d = dev["results"].device
    rows = torch.empty(max(ng, 1) * pw.GENOME_ROW, dtype=torch.uint8, device=d)
    g = torch.from_numpy(np.ascontiguousarray(gof if n else np.zeros(1, np.uint32)).view(np.int32)).to(d)
    ta = torch.from_numpy(np.ascontiguousarray(taln if n else np.zeros(1, np.int32))).to(d)
    return rows[: ng * pw.GENOME_ROW], names, (g, ta, n, ng)


def launch_genome_table(dev, rows, gt, stream_ptr):
    import pwasm_amd as pw
    g, ta, n, ng = gt
    rc = pw.lib().pw_genome_table(dev["results"].data_ptr(), g.data_ptr(), ta.data_ptr(), n,
                                  rows.data_ptr() if ng else 0, ng, stream_ptr)
    if rc != 0:
        raise RuntimeError(f"pw_genome_table: {rc}")


def write_genome_table(path, all_rows, all_names):
    """TSV: target, alignments, event lines, aligned target bases (ranks' rows concatenated; the
    shards are disjoint by construction)."""
    with open(path, "w") as f:
        f.write("#target\talignments\tevents\taligned_bases\n")
        for rows, names in zip(all_rows, all_names):
            r = rows.view(np.uint8).reshape(-1, 16) if rows.size else np.zeros((0, 16), np.uint8)
            rec = r[:, 0:4].copy().view("<u4").ravel()
            ev = r[:, 4:8].copy().view("<u4").ravel()
            tb = r[:, 8:16].copy().view("<u8").ravel()
            for k, nm in enumerate(names):
                f.write(f"{nm.decode()}\t{rec[k]}\t{ev[k]}\t{tb[k]}\n")


def _coll(t, backend):
    """A tensor where the process group's backend wants it (gloo: host)."""
    return t.cpu() if backend == "gloo" else t


def exchange(paf, world, rank, device, backend):
    """Rank r reads only bytes [r*S/N, (r+1)*S/N) of the PAF (pw_paf_split: the lines starting
    there), routes each line to the rank owning its target genome and receives its own lines from
    every rank (all_to_all_single of the bytes and of the global line numbers; over RCCL with the
    nccl backend).  -> (text uint8 with '\\n'-ended lines, global lines uint64, lines in the file)."""
    import torch
    import torch.distributed as dist

    import pwasm_amd as pw
    size = os.path.getsize(paf)
    lo, hi = size * rank // world, size * (rank + 1) // world
    n_local, data, idx = pw.paf_split(paf, lo, hi, world)
    if world == 1:
        return data[0], idx[0].astype(np.uint64), n_local
    dv = device if backend != "gloo" else "cpu"
    cnt = _coll(torch.tensor([n_local], dtype=torch.int64, device=dv), backend)
    counts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(c.item()) for c in counts]
    base = sum(counts[:rank])
    sizes = torch.tensor([[d.size for d in data], [i.size for i in idx]], dtype=torch.int64, device=dv)
    rsizes = torch.empty_like(sizes)
    dist.all_to_all_single(rsizes.view(-1), sizes.t().contiguous().view(-1), [2] * world, [2] * world)
    rsizes = rsizes.view(world, 2).cpu().numpy()
    sb, sl = [d.size for d in data], [i.size for i in idx]
    rb, rl = [int(x) for x in rsizes[:, 0]], [int(x) for x in rsizes[:, 1]]
    send = torch.from_numpy(np.concatenate(data) if sum(sb) else np.zeros(0, np.uint8)).to(dv)
    recv = torch.empty(sum(rb), dtype=torch.uint8, device=dv)
    dist.all_to_all_single(recv, send, rb, sb)
    lines = np.concatenate(idx).astype(np.int64) + base if sum(sl) else np.zeros(0, np.int64)
    sendl = torch.from_numpy(lines).to(dv)
    recvl = torch.empty(sum(rl), dtype=torch.int64, device=dv)
    dist.all_to_all_single(recvl, sendl, rl, sl)
    return recv.cpu().numpy(), recvl.cpu().numpy().astype(np.uint64), sum(counts)


def batch_cuts(text, line_no, target):
    """Sub-batches of at most `target` bytes (at least one line) ending at line ends -> [(byte lo,
    hi, line lo, hi)] (pw_batch_cuts: memchr scans, lines counted by host threads; numpy's
    flatnonzero over the whole text took 0.8 s at cfg3)."""
    import pwasm_amd as pw
    text = np.ascontiguousarray(text)
    if text.dtype != np.uint8:
        raise TypeError("batch_cuts: text must be uint8")
    n = int(text.size)
    if n == 0:
        return []
    cap = n // max(int(target), 1) + 2
    while True:
        out = np.zeros(4 * cap, dtype=np.uint64)
        k = int(pw.lib().pw_batch_cuts(text.ctypes.data, n, max(int(target), 1), out.ctypes.data, cap))
        if k:
            return [tuple(int(x) for x in out[4 * i:4 * i + 4]) for i in range(k)]
        cap *= 4  # (lines longer than target: more batches than n / target)


class OffsetWriter:
    """Output of this rank's finished batches, window by window of global input lines, without a
    merge pass and without holding a rank's whole report: a batch is handed over (add) as soon as
    its outputs are on the host, and each window [j*W, (j+1)*W) is written once every rank has the
    items of all its lines below the window's end (advance).  Per window, in the same order on
    every rank: the first fatal line of the window over all ranks (all-reduce MIN; an input error of
    any rank ends the run too), the per-line stdout byte counts of the window (one owner per line;
    all-reduce SUM of W int64) exclusive-scanned into file offsets after the previous windows, each
    rank's pwrite of its own items there (pw_batch_write_range), stderr gathered to rank 0 only and
    written in line order.  A batch is released once its last item is written: a rank holds every
    batch with a line in the current window or a later one (a batch whose lines reach into later
    windows stays pending until those are written), and each window's collectives make a rank wait
    for the slowest rank to cover that window.  stdout without
    -o: the file is assembled in a temporary file and rank 0 streams each window out after it."""

    BIG = np.iinfo(np.int64).max

    def __init__(self, n_total, out_path, world, rank, dv, tmpdir=None, window=None):
        import torch.distributed as dist
        self.n_total, self.world, self.rank, self.dv = int(n_total), world, rank, dv
        self.W = max(1, int(window or os.environ.get("PW_WINDOW_LINES", str(1 << 21))))
        self.nwin = -(-self.n_total // self.W)
        self.j, self.base, self.code, self.done, self.err = 0, 0, 0, False, None
        self.failed = False  # an input error of some rank, all-reduced: the same on every rank
        self.fatal = False  # the run ended at a fatal line (all-reduced window stop: the same on every rank)
        # world > 1: "exchange" (each rank writes one contiguous range of each window, _exchange_write)
        # or "pwrite" (each rank pwrites its own items at their offsets); PW_MGPU_WRITE picks
        self.mode = os.environ.get("PW_MGPU_WRITE", "exchange")
        self.pending = []  # [[(b, text_h, res_h, pages_h, items), next item, release], ...] in line order
        self.tmp_out = None
        if out_path is None:  # stdout: assembled in a file, streamed out by rank 0 window by window
            if rank == 0:
                fd0, self.tmp_out = tempfile.mkstemp(prefix="pwmg_out_", dir=tmpdir)
                os.close(fd0)
            if world > 1:
                o = [self.tmp_out]
                dist.broadcast_object_list(o, src=0)
                self.tmp_out = o[0]
            out_path = self.tmp_out
        if rank == 0:
            os.close(os.open(out_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644))
        if world > 1:
            dist.barrier()
        self.fd = os.open(out_path, os.O_WRONLY)
        self.rd = open(self.tmp_out, "rb") if self.tmp_out and rank == 0 else None
        self.prof = _Phases(rank, "window")  # PW_PROFILE_HOST: the steps of _window, summed
        self._hb = [None, None]  # exchange write: reused send / receive buffers (_hostbuf)

    def _reduce(self, vals, op):
        import torch
        import torch.distributed as dist
        t = torch.tensor(vals, dtype=torch.int64, device=self.dv)
        if self.world > 1:
            dist.all_reduce(t, op=op)
        return t.cpu().numpy()

    def add(self, out, release=None):
        """A finished batch's outputs; release() is called once all its items are written (the
        host text buffer goes back to its pool)."""
        self.pending.append([out, 0, release])

    def advance(self, covered):
        """This rank has the items of all its lines < covered (n_total: all it will ever have)."""
        while not self.done and self.j < self.nwin and min((self.j + 1) * self.W, self.n_total) <= covered:
            self._window()

    def _window(self):
        import torch
        import torch.distributed as dist
        lo, hi = self.j * self.W, min((self.j + 1) * self.W, self.n_total)
        self.prof.mark("(outside)")
        fatal = self.BIG
        for ent in self.pending:
            (_, _, _, _, (ln, st, _, _)), c = ent[0], ent[1]
            sel = (ln[c:] < hi) & (st[c:] >= 0)
            if sel.any():
                fatal = min(fatal, int(ln[c:][sel][0]))
        MIN = dist.ReduceOp.MIN if self.world > 1 else None
        stop, ok = (int(x) for x in self._reduce([fatal, 0 if self.err else 1], MIN))
        self.prof.mark("stop reduce")
        if not ok:  # an input error on some rank: the first one in rank order, printed by rank 0
            errs = [self.err]
            if self.world > 1:
                errs = [None] * self.world if self.rank == 0 else None
                dist.gather_object(self.err, errs, dst=0)
            if self.rank == 0:
                e = next(x for x in errs if x)
                sys.stderr.write(e.split(": ", 1)[-1] if e.startswith("pw_batch_from_buffer") else e)
                sys.stderr.flush()
            self.code, self.done, self.failed = 1, True, True
            return
        # per line of the window: its stdout bytes * 256 + (owner rank + 1), summed over the ranks (one
        # owner per line): the byte counts, and the owners the exchange write needs
        lens = np.zeros(hi - lo, dtype=np.int64)
        spans, owner = [], -1
        for ent in self.pending:
            (_, _, _, _, (ln, st, on, en)), c = ent[0], ent[1]
            k = c + int(np.searchsorted(ln[c:], min(hi, stop + 1) if stop != self.BIG else hi, side="left"))
            spans.append((c, k))
            if k > c and int(ln[k - 1]) == stop:
                owner = int(st[k - 1])
            lens[ln[c:k].astype(np.int64) - lo] = on[c:k].astype(np.int64) * 256 + (self.rank + 1)
        if self.world > 1:
            tl = torch.from_numpy(lens).to(self.dv)
            dist.all_reduce(tl, op=dist.ReduceOp.SUM)
            lens = tl.cpu().numpy()
        own = (lens & 255).astype(np.int64) - 1  # (-1: a line no rank has an item for)
        lens >>= 8
        off = np.empty(hi - lo + 1, dtype=np.int64)
        off[0] = self.base
        np.cumsum(lens, out=off[1:])
        off[1:] += self.base
        self.prof.mark("offsets")
        errs = []
        exch = self.world > 1 and self.mode == "exchange"
        if exch:  # this rank's items of the window, rendered back to back (line order) into one send buffer
            nbs = [int(ent[0][4][2][c:k].sum()) for ent, (c, k) in zip(self.pending, spans)]
            sbuf = self._hostbuf(0, sum(nbs))
            pos = 0
        for i_ent, (ent, (c, k)) in enumerate(zip(self.pending, spans)):
            if k == c:
                continue
            b, text_h, res_h, pages_h, (ln, st, on, en) = ent[0]
            if exch:
                nb = nbs[i_ent]
                _, eb = b.render_range(text_h, res_h, pages_h, c, nb, k - c, int(en[c:k].sum()),
                                       out=sbuf.numpy()[pos:pos + nb])
                pos += nb
            else:
                eb = b.write_range(text_h, res_h, pages_h, self.fd, c, off[ln[c:k].astype(np.int64) - lo],
                                   int(en[c:k].sum()))
            nz = c + np.flatnonzero(en[c:k])  # (items with stderr bytes: few, a Python loop over them only)
            ends = np.cumsum(en[nz].astype(np.int64))
            for i, e1, n in zip(nz, ends, en[nz]):
                errs.append((int(ln[i]), eb[int(e1) - int(n):int(e1)]))
            ent[1] = k
        self.prof.mark("render/write")
        if exch:
            self._exchange_write(lens, own, off, sbuf[:pos])
        keep = []
        for e in self.pending:
            if e[1] < len(e[0][4][0]):
                keep.append(e)
            elif e[2] is not None:
                e[2]()
        self.pending = keep
        self.prof.mark("exchange write/drop")
        if self.world > 1:  # (every rank's pwrites are done once rank 0 has its stderr)
            allerr = [None] * self.world if self.rank == 0 else None
            dist.gather_object(errs, allerr, dst=0)
            if self.rank == 0:
                errs = sorted((x for e in allerr for x in e), key=lambda t: t[0])
        if self.rd is not None:
            left = int(off[-1]) - self.base
            while left > 0:
                blk = self.rd.read(min(left, 1 << 24))
                if not blk:
                    raise RuntimeError("mgpu: report window shorter than its offsets")
                sys.stdout.buffer.write(blk)
                left -= len(blk)
            sys.stdout.buffer.flush()
        if self.rank == 0:
            for _, e in errs:
                sys.stderr.buffer.write(e)
            sys.stderr.buffer.flush()
        self.prof.mark("stderr/stdout")
        self.base = int(off[-1])
        self.j += 1
        if stop != self.BIG:  # the exit code is the fatal item's (its owner's status)
            self.code = int(self._reduce([owner], dist.ReduceOp.MAX if self.world > 1 else None)[0])
            self.done = True
            self.fatal = True

    def _hostbuf(self, i, n):
        """Reused host buffer i (0: the rendered items sent, 1: the bytes received) of at least n
        bytes, as a uint8 tensor slice: pinned when the collectives run on the GPU (the copies to and
        from the device then need no staging), grown by a quarter when short."""
        import torch
        n = int(n)
        t = self._hb[i]
        if t is None or t.numel() < max(n, 1):
            self._hb[i] = None
            pin = str(self.dv) != "cpu" and torch.cuda.is_available()
            t = self._hb[i] = torch.empty(max(n + n // 4, 1 << 20), dtype=torch.uint8, pin_memory=pin)
        return t[:n]

    def _exchange_write(self, lens, own, off, sbuf):
        """Exchange write of one window (world > 1): the window's bytes are cut into one contiguous
        range per rank at line boundaries; every rank sends each of its rendered items to the rank
        whose range holds it (all_to_all_single: RCCL over xGMI with the nccl backend), and each
        rank writes its whole range with large pwrites (pw_gather_write) — instead of one pwrite per
        item, which serialised the ranks on the output file's inode lock (a rank's lines are
        interleaved with every other rank's: lines are routed by target genome)."""
        import torch
        import torch.distributed as dist

        import pwasm_amd as pw
        n, W, r = len(lens), self.world, self.rank
        start = off[:-1] - off[0]
        total = int(off[-1] - off[0])
        cut = np.searchsorted(start, [total * q // W for q in range(W)], side="left").astype(np.int64)
        cut = np.append(cut, n)
        cut[0] = 0
        idx = np.flatnonzero(own == r)
        dest = np.searchsorted(cut[1:], idx, side="right")
        send = np.bincount(dest, weights=lens[idx], minlength=W).astype(np.int64)
        a, z = int(cut[r]), int(cut[r + 1])
        rng = a + np.flatnonzero(lens[a:z] > 0)
        o_r = own[rng]
        recv = np.bincount(o_r, weights=lens[rng], minlength=W).astype(np.int64)
        if sbuf.numel() != int(send.sum()):
            raise RuntimeError("mgpu: rendered window bytes disagree with the item counts")
        nr = int(recv.sum())
        st = sbuf.to(self.dv, non_blocking=True)  # (gloo: the host tensor itself)
        rt = torch.empty(nr, dtype=torch.uint8, device=self.dv)
        dist.all_to_all_single(rt, st, [int(x) for x in recv], [int(x) for x in send])
        if rt.device.type == "cpu":
            got = rt.numpy()
        else:  # into the reused (pinned) receive buffer; the copy waits for the collective
            rb = self._hostbuf(1, nr)
            rb.copy_(rt)
            got = rb.numpy()
        if rng.size:
            l_r = lens[rng]
            base = np.concatenate([[0], np.cumsum(recv)[:-1]])
            src = np.empty(rng.size, dtype=np.int64)
            for q in range(W):  # (a source's items arrive in line order)
                m = o_r == q
                lq = l_r[m]
                src[m] = base[q] + np.cumsum(lq) - lq
            pw.gather_write(self.fd, int(off[a]), got, src, l_r)

    def close(self):
        """Finish every window; -> the exit code of the single-process run."""
        self.advance(self.n_total)
        self.prof.report()
        os.close(self.fd)
        if self.rd is not None:
            self.rd.close()
        if self.tmp_out and self.rank == 0:
            os.remove(self.tmp_out)
        return self.code


def write_items_at(outs, n_total, out_path, world, rank, dv, tmpdir=None, window=None):
    """All of this rank's finished batches at once through OffsetWriter (tests, small runs).
    Returns the exit code of the single-process run."""
    w = OffsetWriter(n_total, out_path, world, rank, dv, tmpdir, window)
    for o in outs:
        w.add(o)
    return w.close()


def main(argv=None) -> int:
    import queue
    import threading

    import torch
    import torch.distributed as dist

    import pwasm_amd as pw

    argv = sys.argv[1:] if argv is None else argv
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # torchrun sets OMP_NUM_THREADS=1 when the caller left it unset: a rank's host work would run on
    # one thread; give each rank its share of the CPUs instead (PW_THREADS, read by the library first)
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)) or 1)
    if lw > 1 and not os.environ.get("PW_THREADS") and os.environ.get("OMP_NUM_THREADS") == "1":
        os.environ["PW_THREADS"] = str(max(1, min(16, len(os.sched_getaffinity(0)) // lw)))
    backend = os.environ.get("PW_DIST_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
    if world > 1 and not dist.is_initialized():
        # c10d / gloo announce their connections on fd 1: keep that off the report (stdout)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend=backend)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    if world > 1:
        backend = dist.get_backend()
    ndev = torch.cuda.device_count()
    if ndev == 0:
        print("pafreport: no HIP device available (this build has no CPU path)", file=sys.stderr)
        return 2
    device = f"cuda:{local % ndev}"
    torch.cuda.set_device(device)
    try:
        opts, nonopt, extra = parse_args(argv)
    except SystemExit as e:
        if rank == 0:
            print(str(e), file=sys.stderr)
        return 1
    if "w" in opts:
        if rank == 0:
            print("Error: -w (MSA output) is not supported by the multi-GPU driver", file=sys.stderr)
        return 1
    fa = opts.get("r", "")
    if not fa or not nonopt:
        if rank == 0:
            print("Error: query FASTA file (-r) and a PAF file are required!", file=sys.stderr)
        return 1
    flags = ((pw.FLAG_G if "G" in opts else 0) | (pw.FLAG_F if "F" in opts else 0) |
             (pw.FLAG_C if "C" in opts else 0) | (pw.FLAG_N if "N" in opts else 0))
    # the batches run through a pw_runner (the CLI's device session: cs strings packed on the GPU,
    # device buffers reused); PW_MGPU_RUNNER=0: staged through torch tensors, host-packed
    use_runner = os.environ.get("PW_MGPU_RUNNER", "1") != "0"
    if use_runner:
        flags |= pw.FLAG_GPU_PACK
    dv = device if backend != "gloo" else "cpu"

    prof = _Phases(rank)
    # ---- 1. read 1/N of the PAF, exchange lines by target genome
    text, line_no, n_total = exchange(nonopt[0], world, rank, device, backend)
    prof.mark("exchange")

    # ---- 2. this rank's lines in pipelined batches: batch k + 1 is packed (host threads, no GIL)
    # while the GPU runs batch k and its outputs come back (as the CLI pipelines its chunks)
    target = int(os.environ.get("PW_CHUNK_BYTES", str(256 << 20)))
    cuts = batch_cuts(text, line_no, target)
    prof.mark("cuts")
    err = None
    made = {}

    def make(k, prev):
        b0, b1, l0, l1 = cuts[k]
        try:
            made[k] = pw.HostBatch.from_buffer(fa, text[b0:b1], line_no[l0:l1], flags, prev)
        except RuntimeError as e:
            made[k] = e

    out_path = opts.get("o") or None
    # (no more text buffers than this rank has batches: at N = 8 a rank has ~2 batches of cfg3)
    hostbufs = HostTextPool(min(int(os.environ.get("PW_MGPU_HOST_SLOTS", "4")), max(1, len(cuts))))
    writer = OffsetWriter(n_total, out_path, world, rank, dv, extra.get("tmpdir"))
    # ---- 3. the writer thread: each finished batch is handed over with the line its rank has
    # covered, and the windows that completes are written (offsets, render + pwrite, stderr) while
    # this thread stages / runs / fetches the next batch.  The writer's collectives (window
    # reductions, the exchange write) are the only ones between exchange() and finish_run, so their
    # order is the same on every rank.
    wq = queue.Queue(maxsize=int(os.environ.get("PW_MGPU_WRITE_QUEUE", "2")))
    werr = []

    def write_loop():
        if device.startswith("cuda"):
            torch.cuda.set_device(device)
        while True:
            job = wq.get()
            if job is None:
                return
            out, release, covered = job
            if werr:
                release()
                continue
            try:
                writer.add(out, release)
                if covered is not None:
                    writer.advance(covered)
            except BaseException as e:  # (re-raised by the main thread)
                werr.append(e)
    wth = threading.Thread(target=write_loop, name="pw-mgpu-writer", daemon=True)
    wth.start()
    stream = torch.cuda.current_stream()
    want_tab = "genome-table" in extra
    gname, gacc = {}, np.zeros((1024, 3), np.uint64)  # target name -> row of the summed per-genome table
    th = None
    runner = None
    if cuts:
        th = threading.Thread(target=make, args=(0, None))
        th.start()
    for k in range(len(cuts)):
        th.join()
        prof.mark("pack wait")
        b = made.pop(k)
        if isinstance(b, RuntimeError):
            err = str(b)
            break
        if k + 1 < len(cuts):
            th = threading.Thread(target=make, args=(k + 1, b))
            th.start()
        slot = []
        dev = None
        if use_runner:
            if runner is None:
                runner = pw.Runner(b)
            npg, used = runner.run(b)  # (GPU cs packing, the pass, results and pages back)
            prof.mark("gpu pack + pass")
            t = hostbufs.take(max(used, 1), slot)
            prof.mark("fetch alloc")
            text_h, res_h, pages_h = runner.fetch(t, npg, used)
            prof.mark("fetch text")
            if want_tab:  # (the per-genome tables only when asked for: --genome-table)
                rows_h, names = runner.genome_rows(b)
        else:
            dev = pw.stage_batch(b, device)
            prof.mark("stage")
            pw.run_report(b, dev, stream.cuda_stream)
            if want_tab:
                rows, names, gt = genome_rows(b, dev, stream.cuda_stream)
                launch_genome_table(dev, rows, gt, stream.cuda_stream)
            if prof.on:
                stream.synchronize()
                prof.mark("gpu pass")

            def take(n):
                prof.mark("fetch results/pages")
                t = hostbufs.take(n, slot)
                prof.mark("fetch alloc")
                return t
            text_h, res_h, pages_h = pw.fetch_outputs(dev, take)  # (synchronises the stream)
            prof.mark("fetch text")
            if want_tab:
                rows_h = rows.cpu().numpy()
        if want_tab:  # per-genome rows of all batches, summed by target (vectorised: 50k targets a batch at cfg3)
            r = rows_h.view(np.uint8).reshape(-1, 16) if len(names) else np.zeros((0, 16), np.uint8)
            gidx = np.fromiter((gname.setdefault(nm, len(gname)) for nm in names), dtype=np.int64, count=len(names))
            if len(gname) > gacc.shape[0]:
                gacc = np.concatenate([gacc, np.zeros((max(len(gname), 2 * gacc.shape[0]) - gacc.shape[0], 3), np.uint64)])
            vals = np.stack([r[:, 0:4].copy().view("<u4").ravel().astype(np.uint64),
                             r[:, 4:8].copy().view("<u4").ravel().astype(np.uint64),
                             r[:, 8:16].copy().view("<u8").ravel()], axis=1) if len(names) else np.zeros((0, 3), np.uint64)
            np.add.at(gacc, gidx, vals)
            prof.mark("genome rows")
        items = b.items(text_h, res_h, pages_h)
        fatal = bool((items[1] >= 0).any())  # a fatal item: nothing after it is reached
        covered = None if fatal else (int(line_no[cuts[k + 1][2]]) if k + 1 < len(cuts) else n_total)
        prof.mark("items")
        wq.put(((b, text_h, res_h, pages_h, items), (lambda i=slot[0]: hostbufs.give(i)), covered))
        del dev, b
        prof.mark("writer queue wait")
        if fatal or werr or writer.done:  # (done: the run ended at a window every rank has processed)
            break
    wq.put(None)
    wth.join()
    prof.mark("writer drain")
    if werr:
        raise werr[0]
    if th is not None and th.is_alive():
        th.join()
    made.clear()
    if runner is not None:
        runner.close()
    gtabs = {nm: gacc[i] for nm, i in gname.items()}
    code = finish_run(writer, err, gtabs, extra, world, rank, device)
    prof.mark("finish")
    prof.report()
    return code


class HostTextPool:
    """Reused pinned host buffers for the batches' report text (fetch_outputs): a fresh pageable
    array per batch cost a page fault per 4 KB on the copy and an unmap of ~1 GB when the batch was
    dropped.  A buffer is busy from take() until its batch's items are all written (give(), called
    by OffsetWriter from the writer thread); when every slot is busy take() falls back to a pageable
    tensor.  The first take() sizes a slot at 1.5x its request and allocates the other slots at that
    size on a helper thread (pinning ~1.5 GB takes ~0.3 s), so later batches find them ready.
    Without a GPU (tests) the buffers are ordinary host memory."""

    def __init__(self, slots=4):
        self.bufs, self.busy = [None] * max(0, slots), [False] * max(0, slots)
        self.pre = None  # the helper thread allocating the other slots

    def _alloc(self, n):
        import torch
        return torch.empty(int(n), dtype=torch.uint8, pin_memory=torch.cuda.is_available())

    def take(self, n, slot_out):
        import threading

        import torch
        n = int(n)
        first = all(b is None for b in self.bufs)
        if not first and self.pre is not None:
            self.pre.join()
            self.pre = None
        free = [i for i, b in enumerate(self.busy) if not b]
        fit = [i for i in free if self.bufs[i] is not None and self.bufs[i].numel() >= n]
        if fit:
            i = fit[0]
        elif free:
            i = free[0]
            cap = n + n // 2 + (1 << 20)
            self.bufs[i] = None  # (release the smaller one first)
            self.bufs[i] = self._alloc(cap)
            if first and len(self.bufs) > 1:
                dev = torch.cuda.current_device() if torch.cuda.is_available() else None

                def pre():  # (on the caller's device: a thread starts on device 0)
                    if dev is not None:
                        torch.cuda.set_device(dev)
                    for j in range(len(self.bufs)):
                        if self.bufs[j] is None:
                            self.bufs[j] = self._alloc(cap)
                self.pre = threading.Thread(target=pre, daemon=True)
                self.pre.start()
        else:  # (pageable: pinning a one-off buffer costs more than its copy saves)
            slot_out.append(None)
            return torch.empty(n, dtype=torch.uint8)
        self.busy[i] = True
        slot_out.append(i)
        return self.bufs[i][:n]

    def give(self, i):
        if i is not None:
            self.busy[i] = False


class _Phases:
    """PW_PROFILE_HOST=1: wall time per phase of main() (summed over batches), one stderr line per rank."""

    def __init__(self, rank, what="rank"):
        import time
        self.on = bool(os.environ.get("PW_PROFILE_HOST"))
        self.rank, self.t, self.acc, self.clock, self.what = rank, time.perf_counter(), {}, time.perf_counter, what

    def mark(self, name):
        if self.on:
            t = self.clock()
            self.acc[name] = self.acc.get(name, 0.0) + t - self.t
            self.t = t

    def report(self):
        if self.on:
            print(f"[mgpu {self.what} {self.rank}] " + ", ".join(f"{k} {v:.3f} s" for k, v in self.acc.items()),
                  file=sys.stderr, flush=True)


def finish_run(writer, err, gtabs, extra, world, rank, device):
    """The end of main() on every rank: the remaining windows, then (unless an input error ended
    the run) the per-genome table all-gather and the final barrier.  The early return keys on
    writer.failed — the error all-reduced over the ranks inside the windows — not on this rank's
    own `err`, so a rank without lines (or whose batches all read fine) takes the same path as the
    rank that failed and no collective is left waiting (tests/test_mgpu_cpu.py)."""
    import torch
    import torch.distributed as dist
    writer.err = err
    code = writer.close()
    # A run that ends at a fatal line writes no genome table: each rank stops at whatever batch it
    # had reached when that line's window completed, so the rows would depend on timing.
    if writer.failed or writer.fatal:
        return code
    if "genome-table" in extra:
        names = list(gtabs.keys())
        rows = (np.stack([gtabs[n] for n in names]) if names else np.zeros((0, 3), np.uint64))
        packed = np.zeros((len(names), 16), np.uint8)
        packed[:, 0:4] = rows[:, 0].astype("<u4").reshape(-1, 1).view(np.uint8)
        packed[:, 4:8] = rows[:, 1].astype("<u4").reshape(-1, 1).view(np.uint8)
        packed[:, 8:16] = rows[:, 2].astype("<u8").reshape(-1, 1).view(np.uint8)
        rt = torch.from_numpy(packed.reshape(-1).copy()).to(device)
        nb = b"\0".join(names)
        nt = torch.from_numpy(np.frombuffer(nb, dtype=np.uint8).copy() if nb else np.zeros(0, np.uint8)).to(device)
        if world > 1:  # (RCCL all-gather of the rows; the names ride along)
            all_rows = [x.cpu().numpy() for x in gather_ragged(rt)]
            all_names = [bytes(x.cpu().numpy()).split(b"\0") if x.numel() else [] for x in gather_ragged(nt)]
        else:
            all_rows, all_names = [rt.cpu().numpy()], [names]
        if rank == 0:
            write_genome_table(extra["genome-table"], all_rows, all_names)
    if world > 1:
        dist.barrier()
    return code


if __name__ == "__main__":
    rc = main()
    try:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:
        pass
    sys.stdout.flush()
    sys.exit(rc)
