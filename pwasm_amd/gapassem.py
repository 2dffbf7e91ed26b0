"""GapAssem column consensus on the HIP path, rows sharded over GPUs.

The single-GPU product is the C++ driver pw_gapassem_run (gapassem_consensus CLI).  This module
is the multi-GPU driver of the same computation, one process per GPU:

  every rank    reads the PWL1 row headers (GASeq offset/seqlen/clp5/clp3/revcompl), derives
                minoffset and the layout length (GSeqAlign bookkeeping, GapAssem.cpp:605-641,
                694-716) and stages ITS rows (a contiguous, base-balanced block) in HBM;
  pw_msa_count  buildMSA's toMSA/addNuc/addGap scatter of those rows -> partial [n_cols x 6]
                int32 histograms + mincol/maxcol (GapAssem.cpp:551-591, 1088-1106);
  collectives   with the "nccl" backend (the product) the column-sharded call of the C-ABI,
  + call        pw_msa_call_sharded on an RCCL communicator of its own (rccl_comm), on the rank's
                stream: a reduce-scatter of the histograms by column range + MIN/MAX of (mincol,
                maxcol, first bad row), bestChar (GapAssem.cpp:1048-1069) and the zero-coverage
                scan of the rank's columns only, an all-gather of the consensus ranges; rank 0
                gathers the column ranges of the histogram for the result file.  Integer sums are
                order-independent: bit-identical to a single-GPU count.  (PW_GA_COMM=rccl-allreduce:
                one all-reduce of the whole histogram + pw_msa_call everywhere; under gloo the
                same through torch.distributed, for rehearsals.)
  pw_msa_refine refineMSA's consensus string and, with removeConsGaps, the closed-form
                removeColumn/removeBase edits of the rank's own rows (GapAssem.cpp:1143-1162);
  finish_rows   the per-row tail on the host through the C-ABI: removeColumn replayed for rows
                with deleted bases, refineClipping, removeClipGaps (GapAssem.cpp:1163-1181).
Rank 0 writes the PWC1 result (edited rows gathered from their owners).  Messages and exit codes
are the reference's (trimmed-row warnings :1096-1101, bad index GapAssem.h:366-370 -> 1, zero
coverage :1121-1131 -> 5), in row order, as the single-GPU driver prints them.

Device work goes through an engine: HipEngine is the product (libpwasm_amd.so on this rank's GPU;
there is no CPU path).  Tests substitute a CPU engine to exercise the collective choreography on
gloo without a GPU."""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

INT_MAX = 2 ** 31 - 1


class Layout:
    """PWL1 rows (tests/pwl_format.md): every row's header; bases/gaps of the rows in `load`
    (None = all)."""

    def __init__(self, path: str, load=None):
        with open(path, "rb") as f:
            b = f.read(8)
            if len(b) < 8 or b[:4] != b"PWL1" or struct.unpack("<I", b[4:8])[0] == 0:
                raise ValueError("bad layout header")
            (n,) = struct.unpack("<I", b[4:8])
            hdr = np.zeros((n, 5), dtype=np.int64)
            numgaps = np.zeros(n, dtype=np.int64)
            self.seq, self.ofs = {}, {}
            for r in range(n):
                h = f.read(20)
                if len(h) < 20:
                    raise ValueError("bad row header")
                hdr[r] = struct.unpack("<5i", h)
                L = int(hdr[r, 1])
                if L < 0:
                    raise ValueError("bad row header")
                seq = f.read(L)
                ofs = np.frombuffer(f.read(2 * L), dtype="<i2")
                if len(seq) != L or ofs.size != L:
                    raise ValueError("truncated row")
                numgaps[r] = int(ofs.sum(dtype=np.int64))  # setGap bookkeeping
                if load is None or r in load:
                    self.seq[r] = np.frombuffer(seq, dtype=np.uint8)
                    self.ofs[r] = ofs.astype(np.int16)
        self.n = n
        self.offset, self.seqlen, self.clp5, self.clp3, self.rev = (hdr[:, i].copy() for i in range(5))
        self.numgaps = numgaps
        self.minoffset = int(self.offset.min())
        self.length = max(int((self.offset + self.seqlen + self.numgaps).max()) - self.minoffset, 0)

    def clips(self, r):
        """clipL / clipR oriented by revcompl (GapAssem.cpp:557-564)."""
        return (int(self.clp3[r]), int(self.clp5[r])) if self.rev[r] else (int(self.clp5[r]), int(self.clp3[r]))


def shard_rows(seqlen, world: int):
    """Contiguous row blocks with about equal bases per rank, every block non-empty when
    world <= rows: [(lo, hi)] per rank."""
    n = len(seqlen)
    cum = np.concatenate([[0], np.cumsum(np.asarray(seqlen, dtype=np.int64))])
    tot = int(cum[-1])
    cuts = [0]
    for k in range(1, world):
        c = int(np.searchsorted(cum, tot * k / world, side="left"))
        c = min(max(c, cuts[-1] + (1 if n >= world else 0)), n - (world - k) if n >= world else n)
        cuts.append(c)
    cuts.append(n)
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


class HipEngine:
    """Device work of one shard through the C-ABI (pw_msa_count / pw_msa_call / pw_msa_refine)."""

    def __init__(self, device: str = "cuda:0"):
        import torch
        from pwasm_amd import lib
        self.torch, self.lib, self.device = torch, lib(), device
        self.stream = torch.cuda.current_stream(device)

    def stage(self, lay: Layout, rows, ncols: int, nranks: int = 1):
        """Stage the rows; nranks > 1: the histograms and consensus padded to nranks column ranges
        of cols_per_rank (the column-sharded call, pw_msa_call_sharded)."""
        from pwasm_amd import MsaArgs, MsaRefineArgs
        torch, dev = self.torch, self.device
        rows = list(rows)
        nr = len(rows)
        if nr == 0:
            raise ValueError("gapassem: a shard without rows")
        lens = np.array([int(lay.seqlen[r]) for r in rows], dtype=np.int32)
        # rows start 8-base aligned (the count kernels' vector loads); the gaps between rows are zero
        padded = (lens.astype(np.uint64) + 7) // 8 * 8
        row_off = np.concatenate([[0], np.cumsum(padded)])[:nr].astype(np.uint64)
        total = int(row_off[-1] + padded[-1]) if nr else 0
        seq = np.zeros(max(total, 1), dtype=np.uint8)
        ofs = np.zeros(max(total, 1), dtype=np.int16)
        for k, r in enumerate(rows):
            o = int(row_off[k])
            seq[o:o + int(lens[k])] = lay.seq[r]
            ofs[o:o + int(lens[k])] = lay.ofs[r]
        cl = np.array([lay.clips(r)[0] for r in rows], dtype=np.int32)
        cr = np.array([lay.clips(r)[1] for r in rows], dtype=np.int32)
        col0 = np.array([int(lay.offset[r]) - lay.minoffset for r in rows], dtype=np.int32)
        slot_base = np.zeros(nr + 1, dtype=np.int64)
        nslots = int(self.lib.pw_msa_slots(lens.ctypes.data, nr, slot_base.ctypes.data))

        def t(a):
            a = np.ascontiguousarray(a)
            if a.size == 0:
                a = np.zeros(1, dtype=a.dtype)
            return torch.from_numpy(a.view(np.uint8) if a.dtype == np.uint64 else a).to(dev)

        def e(n, dt):
            return torch.empty(max(int(n), 1), dtype=dt, device=dev)

        cpr = (ncols + nranks - 1) // nranks
        d = {"seq": t(seq), "ofs": t(ofs), "row_off": t(row_off), "len": t(lens), "col0": t(col0), "cl": t(cl),
             "cr": t(cr), "slot": t(slot_base), "scr": e(self._scratch_words(nslots, nr), torch.int32),
             "counts": torch.zeros(max(nranks * cpr * 6, 1), dtype=torch.int32, device=dev),
             "cons": torch.zeros(max(nranks * cpr, 1), dtype=torch.uint8, device=dev), "mm": e(4, torch.int32),
             "cpart": e(cpr * 6, torch.int32),
             "gp": e(ncols, torch.int32), "tg": e(self.lib.pw_msa_refine_tiles(ncols), torch.int32),
             "cout": e(ncols, torch.uint8), "clen": e(1, torch.int32),
             "roffs": t(np.array([int(lay.offset[r]) for r in rows], dtype=np.int32)),
             "ofso": e(ofs.size, torch.int16), "offo": e(nr, torch.int32), "ngo": e(nr, torch.int64),
             "ng0": t(np.array([int(lay.numgaps[r]) for r in rows], dtype=np.int64))}
        a = MsaArgs()
        a.seq, a.ofs, a.row_off, a.row_len = (d[k].data_ptr() for k in ("seq", "ofs", "row_off", "len"))
        a.col0, a.clip_l, a.clip_r, a.slot_base = (d[k].data_ptr() for k in ("col0", "cl", "cr", "slot"))
        a.scratch, a.counts, a.consensus, a.minmax = (d[k].data_ptr() for k in ("scr", "counts", "cons", "mm"))
        a.n_slots, a.n_rows, a.n_cols = nslots, nr, ncols
        ra = MsaRefineArgs()
        ra.keep_clip_gaps = 1  # refineClipping / removeClipGaps per row on the host (finish_rows)
        ra.gap_prefix, ra.tile_gaps, ra.cons_out, ra.cons_len = (d[k].data_ptr() for k in ("gp", "tg", "cout", "clen"))
        ra.row_offset, ra.ofs_out, ra.offset_out, ra.numgaps_out = (d[k].data_ptr()
                                                                    for k in ("roffs", "ofso", "offo", "ngo"))
        return dict(rows=rows, nr=nr, lens=lens, row_off=row_off, ncols=ncols, d=d, args=a, rargs=ra, cpr=cpr)

    def _scratch_words(self, nslots: int, nr: int) -> int:
        f = getattr(self.lib, "pw_msa_scratch_words", None)
        return int(f(nslots, nr)) if f is not None else 3 * nslots  # (older experiment builds)

    def _rc(self, name, rc):
        if rc != 0:
            raise RuntimeError(f"{name}: {rc}")

    def count(self, st):
        """-> (counts [ncols*6] int32, minmax [4] int32) device tensors; minmax[2] = first bad
        row of this shard (local index) or INT_MAX."""
        self._rc("pw_msa_count", self.lib.pw_msa_count(ctypes.byref(st["args"]), self.stream.cuda_stream))
        return st["d"]["counts"], st["d"]["mm"]

    def columns(self, st):
        """count + call of a single shard in one pass (pw_msa_columns: bestChar from tile_counts'
        complete per-tile counts) -> (counts, minmax); the consensus is st["d"]["cons"]."""
        self._rc("pw_msa_columns", self.lib.pw_msa_columns(ctypes.byref(st["args"]), self.stream.cuda_stream))
        return st["d"]["counts"], st["d"]["mm"]

    def merge(self, st, row_base: int, comm):
        """pw_msa_counts_allreduce over an RCCL communicator (rccl_comm): histograms summed,
        bounds reduced, the bad row made global — in place on every rank."""
        self._rc("pw_msa_counts_allreduce", self.lib.pw_msa_counts_allreduce(ctypes.byref(st["args"]), row_base, comm,
                                                                             self.stream.cuda_stream))
        return st["d"]["counts"], st["d"]["mm"]

    def call_sharded(self, st, row_base: int, comm, rank: int, nranks: int):
        """pw_msa_call_sharded: histograms reduce-scattered by column range over RCCL, bestChar of
        this rank's range, the consensus all-gathered -> (consensus, minmax, this range's counts)."""
        self._rc("pw_msa_call_sharded", self.lib.pw_msa_call_sharded(ctypes.byref(st["args"]), row_base,
                                                                     st["d"]["cpart"].data_ptr(), st["cpr"], rank,
                                                                     nranks, comm, self.stream.cuda_stream))
        return st["d"]["cons"], st["d"]["mm"], st["d"]["cpart"]

    def call(self, st):
        """bestChar per column + first zero-coverage column (minmax[3]) from the merged counts."""
        self._rc("pw_msa_call", self.lib.pw_msa_call(ctypes.byref(st["args"]), self.stream.cuda_stream))
        return st["d"]["cons"], st["d"]["mm"]

    def columns_refine(self, st, remove_gaps: bool):
        """columns + refine of a single shard holding every row (pw_msa_columns_refine: without
        removeConsGaps the consensus string comes out of the counting pass)."""
        d, ra = st["d"], st["rargs"]
        ra.remove_gaps = 1 if remove_gaps else 0
        if remove_gaps:
            d["ngo"].copy_(d["ng0"])
        self._rc("pw_msa_columns_refine", self.lib.pw_msa_columns_refine(ctypes.byref(st["args"]), ctypes.byref(ra),
                                                                         self.stream.cuda_stream))
        return d["counts"], d["mm"]

    def refine(self, st, remove_gaps: bool):
        """Launch pw_msa_refine (device results stay in st["d"])."""
        d, ra = st["d"], st["rargs"]
        ra.remove_gaps = 1 if remove_gaps else 0
        if remove_gaps:
            d["ngo"].copy_(d["ng0"])
        self._rc("pw_msa_refine", self.lib.pw_msa_refine(ctypes.byref(st["args"]), ctypes.byref(ra),
                                                         self.stream.cuda_stream))

    def refine_host(self, st, remove_gaps: bool):
        """-> (consensus bytes, {row: (offset, numgaps, ofs)} for own rows when remove_gaps)."""
        self.refine(st, remove_gaps)
        d = st["d"]
        clen = int(d["clen"].cpu().item())
        cons = bytes(d["cout"][:clen].cpu().numpy())
        rows = {}
        if remove_gaps:
            offo, ngo, ofso = d["offo"].cpu().numpy(), d["ngo"].cpu().numpy(), d["ofso"].cpu().numpy()
            for k, r in enumerate(st["rows"]):
                o = int(st["row_off"][k])
                rows[r] = (int(offo[k]), int(ngo[k]), ofso[o:o + int(st["lens"][k])].copy())
        return cons, rows


_COMMS = {}


def rccl_comm(group=None):
    """An RCCL communicator over the ranks of `group` for the C-ABI collectives (one per group,
    kept for the process): rank 0 draws the id, torch.distributed broadcasts it."""
    import torch.distributed as dist
    from pwasm_amd import lib
    key = id(group)
    if key in _COMMS:
        return _COMMS[key]
    L = lib()
    buf = ctypes.create_string_buffer(128)
    if dist.get_rank(group) == 0 and L.pw_comm_unique_id(buf) != 0:
        raise RuntimeError("pw_comm_unique_id")
    obj = [buf.raw]
    dist.broadcast_object_list(obj, src=0, group=group)
    buf = ctypes.create_string_buffer(obj[0], 128)
    comm = ctypes.c_void_p()
    if L.pw_comm_init(ctypes.byref(comm), dist.get_world_size(group), buf, dist.get_rank(group)) != 0:
        raise RuntimeError("pw_comm_init")
    _COMMS[key] = comm
    return comm


def all_reduce(t, op, group=None):
    """dist.all_reduce; device tensors under gloo (CPU-only collectives) go through the host."""
    import torch.distributed as dist
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)


def _bad_index_col(lay: Layout, r: int, ncols: int):
    """First column toMSA touches out of range for row r (GapAssem.cpp:568-588)."""
    cl, cr = lay.clips(r)
    col = int(lay.offset[r]) - lay.minoffset
    L = int(lay.seqlen[r])
    for i, g in enumerate(lay.ofs[r].tolist()):
        clipped = i < cl or i >= L - cr
        for _ in range(g):
            if not clipped and (col < 0 or col >= ncols):
                return col
            col += 1
        if col < 0 or col >= ncols:
            return col
        col += 1
    return None


def _i32(v: int) -> int:
    """int32 wrap-around (the reference's int arithmetic)."""
    return (v + 2 ** 31) % 2 ** 32 - 2 ** 31


def finish_rows(lay: Layout, rows, base: dict, alpos, cons: bytes, mincol: int, remove_gaps: bool,
                refine_clipping: bool, msg_cap: int = 1 << 16):
    """refineMSA's per-row tail for `rows` on the host (GapAssem.cpp:1163-1181), all rows in one
    C call (pw_ga_rows_finish): rows holding deleted bases (ofs < 0) get removeColumn replayed from
    their input gaps, every row then refineClipping / removeClipGaps / refineClipping.  base =
    {row: (offset, numgaps, ofs)} after the GPU's removeColumn edits.  Stops after a row that
    GErrors (the reference exits there).  -> {row: (messages, failed, offset, numgaps, clp5,
    clp3, ofs)} for the rows processed."""
    from pwasm_amd import GaRow, lib
    rows = list(rows)
    n = len(rows)
    if n == 0:
        return {}
    L = lib()
    flags = (1 if remove_gaps else 0) | (2 if refine_clipping else 0)
    al = np.ascontiguousarray(np.asarray(alpos, dtype=np.int32))
    cons_a = np.frombuffer(cons, dtype=np.uint8) if cons else np.zeros(1, dtype=np.uint8)
    replay = np.array([remove_gaps and int(lay.ofs[r].min(initial=0)) < 0 for r in rows], dtype=np.uint8)
    lens = np.array([int(lay.seqlen[r]) for r in rows], dtype=np.int64)
    start = np.concatenate([[0], np.cumsum(lens)])
    seq = np.concatenate([np.asarray(lay.seq[r], dtype=np.uint8) for r in rows] + [np.zeros(1, np.uint8)])
    ofs = np.concatenate([np.asarray(lay.ofs[r] if replay[k] else base[r][2], dtype=np.int16)
                          for k, r in enumerate(rows)] + [np.zeros(1, np.int16)])
    off0 = np.array([int(lay.offset[r]) if replay[k] else int(base[r][0]) for k, r in enumerate(rows)], np.int64)
    ng0 = np.array([int(lay.numgaps[r]) if replay[k] else int(base[r][1]) for k, r in enumerate(rows)], np.int64)
    ids = b"".join(b"row%d\0" % r for r in rows)
    id_off = np.concatenate([[0], np.cumsum([len(b"row%d" % r) + 1 for r in rows])])[:n]
    idbuf = ctypes.create_string_buffer(ids, len(ids))
    arr = (GaRow * n)()
    dt = np.dtype({"names": ["seq", "ofs", "seqlen", "offset", "numgaps", "clp5", "clp3", "rev", "id"],
                   "formats": ["<u8", "<u8", "<i4", "<i4", "<i4", "<i4", "<i4", "<i4", "<u8"],
                   "offsets": [GaRow.seq.offset, GaRow.ofs.offset, GaRow.seqlen.offset, GaRow.offset.offset,
                               GaRow.numgaps.offset, GaRow.clp5.offset, GaRow.clp3.offset, GaRow.revcompl.offset,
                               GaRow.id.offset], "itemsize": ctypes.sizeof(GaRow)})
    v = np.frombuffer(arr, dtype=dt)
    ri = np.array(rows, dtype=np.int64)
    v["seq"] = seq.ctypes.data + start[:n]
    v["ofs"] = ofs.ctypes.data + 2 * start[:n]
    v["seqlen"] = lens
    v["offset"] = off0
    v["numgaps"] = ng0
    v["clp5"] = lay.clp5[ri]
    v["clp3"] = lay.clp3[ri]
    v["rev"] = lay.rev[ri]
    v["id"] = ctypes.addressof(idbuf) + id_off
    cap = max(1, int(msg_cap))
    while True:  # an overflowing call leaves every row as it was (pw_ga_rows_finish restores them)
        msg = ctypes.create_string_buffer(cap)
        moff = np.zeros(n + 1, dtype=np.uint64)
        failed = np.zeros(n, dtype=np.int32)
        k = L.pw_ga_rows_finish(arr, n, replay.ctypes.data, al.ctypes.data if al.size else None, al.size,
                                cons_a.ctypes.data, len(cons), _i32(lay.minoffset + mincol), flags, msg, cap,
                                moff.ctypes.data, failed.ctypes.data)
        if k < 0:
            raise RuntimeError(f"pw_ga_rows_finish: {k}")
        if int(moff[k]) <= cap:
            break
        cap = int(moff[k])
    raw = msg.raw
    out = {}
    for j in range(int(k)):
        out[rows[j]] = (raw[int(moff[j]):int(moff[j + 1])].decode(), bool(failed[j]), int(v["offset"][j]),
                        int(v["numgaps"][j]), int(v["clp5"][j]), int(v["clp3"][j]),
                        ofs[int(start[j]):int(start[j + 1])].copy())
    return out


def gather_rows(fin: dict, group, device):
    """finish_rows' output of every rank, merged on rank 0 only (the one that writes the result;
    None elsewhere).  The per-row fields (messages, offsets, clips: small) go through
    gather_object; the edited gap arrays (all rows with removeConsGaps: ~2 bytes per base) as one
    byte tensor per rank through gather — device tensors under RCCL (int16 is not an RCCL type:
    the bytes travel), host tensors under gloo."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    rows = sorted(fin)
    meta = {r: fin[r][:6] + (len(fin[r][6]),) for r in rows}
    flat = (np.concatenate([np.asarray(fin[r][6], dtype="<i2") for r in rows]) if rows
            else np.zeros(0, dtype="<i2")).view(np.uint8)
    metas = [None] * world if rank == 0 else None
    dist.gather_object((meta, int(flat.size)), metas, dst=0, group=group)
    nmax = torch.tensor([int(flat.size)], dtype=torch.int64)
    dev = device if dist.get_backend(group) == "nccl" else "cpu"
    nmax = nmax.to(dev)
    dist.all_reduce(nmax, op=dist.ReduceOp.MAX, group=group)
    nmax = max(1, int(nmax.item()))
    buf = torch.zeros(nmax, dtype=torch.uint8, device=dev)
    if flat.size:
        buf[: flat.size] = torch.from_numpy(flat).to(dev)
    outs = [torch.empty(nmax, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, outs, dst=0, group=group)
    if rank != 0:
        return None
    merged = {}
    for (meta_p, n), t in zip(metas, outs):
        b = t[:n].cpu().numpy().view("<i2") if n else np.zeros(0, dtype="<i2")
        o = 0
        for r in sorted(meta_p):
            m = meta_p[r]
            merged[r] = m[:6] + (b[o: o + m[6]].astype(np.int16),)
            o += m[6]
    return merged


def consensus(layout_path: str, remove_gaps: bool = False, group=None, engine=None, refine_clipping: bool = True):
    """refineMSA's consensus with rows sharded over the ranks of `group` (torch.distributed; a
    single process when it is not initialised).  Returns (exit_code, stderr_text, pwc_bytes) on
    rank 0 — the same bytes as the gapassem_consensus CLI — and (exit_code, "", None) elsewhere."""
    import torch
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if dist_on else 1
    rank = dist.get_rank(group) if dist_on else 0
    hdr = Layout(layout_path, load=set())
    lo, hi = shard_rows(hdr.seqlen, world)[rank]
    lay = Layout(layout_path, load=set(range(lo, hi)))
    ncols = lay.length
    if ncols <= 0 or ncols > INT_MAX:
        return 1, ("MSAColumns op[]: bad index 0 (size=%d)\n" % ncols) if rank == 0 else "", None
    engine = engine or HipEngine()
    mode = os.environ.get("PW_GA_COMM", "auto")  # auto | rccl / rccl-allreduce (also at world 1) | torch
    use_rccl = (dist_on and isinstance(engine, HipEngine) and dist.get_backend(group) == "nccl"
                and (mode in ("rccl", "rccl-allreduce") or (mode == "auto" and world > 1)))
    sharded = use_rccl and mode != "rccl-allreduce"  # column-sharded call (reduce-scatter + all-gather)
    st = engine.stage(lay, range(lo, hi), ncols, world if sharded else 1)
    fused = world == 1 and not use_rccl and hasattr(engine, "columns")  # (one shard: count + call in one pass)
    counts, mm = engine.columns(st) if fused else engine.count(st)
    mm_h = [int(x) for x in mm.cpu().tolist()]
    called = (st["d"]["cons"], mm) if fused else None
    if sharded:  # pw_msa_call_sharded: reduce-scatter by column range, own-range bestChar, all-gather
        cons_cols, mm, part = engine.call_sharded(st, lo, rccl_comm(group), rank, world)
        called = (cons_cols, mm)
        mm_h = [int(x) for x in mm.cpu().tolist()]
        bad = mm_h[2]
        mm_h[2] = INT_MAX
        # the full histogram for the result file, on rank 0 only
        parts = [torch.empty_like(part) for _ in range(world)] if rank == 0 else None
        dist.gather(part, parts, dst=0, group=group)
        if rank == 0:
            counts = torch.cat(parts)[: ncols * 6]
    elif use_rccl:  # the C-ABI all-reduce (pw_msa_counts_allreduce) on this rank's stream
        counts, mm = engine.merge(st, lo, rccl_comm(group))
        mm_h = [int(x) for x in mm.cpu().tolist()]
        bad = mm_h[2]
        mm_h[2] = INT_MAX
    else:
        bad = lo + mm_h[2] if mm_h[2] != INT_MAX else INT_MAX
    if world > 1 and not use_rccl:
        red = torch.tensor([mm_h[0], -mm_h[1], bad], dtype=torch.int64, device=counts.device)
        all_reduce(counts, dist.ReduceOp.SUM, group)
        all_reduce(red, dist.ReduceOp.MIN, group)
        red = [int(x) for x in red.cpu().tolist()]
        mm_h[0], mm_h[1], bad = red[0], -red[1], red[2]
        mm.copy_(torch.tensor([mm_h[0], mm_h[1], INT_MAX, INT_MAX], dtype=torch.int32))
    err = []
    for r in range(min(hdr.n if bad == INT_MAX else bad + 1, hdr.n)):
        if int(lay.seqlen[r] - lay.clp3[r] - lay.clp5[r]) < 1:
            err.append("Warning: sequence row%u (length %d) was trimmed too badly (%d,%d) -- should be removed from "
                       "MSA w/ row0!\n" % (r, lay.seqlen[r], lay.clp5[r], lay.clp3[r]))
    if bad != INT_MAX:
        col = _bad_index_col(lay, bad, ncols) if lo <= bad < hi else None
        if world > 1:
            cols = [None] * world
            dist.all_gather_object(cols, col, group=group)
            col = next(c for c in cols if c is not None)
        err.append("MSAColumns op[]: bad index %d (size=%d)\n" % (col, ncols))
        return 1, "".join(err) if rank == 0 else "", None
    cons_cols, mm = called if called else engine.call(st)
    zero = int(mm[3].item())
    mincol, maxcol = mm_h[0], max(mm_h[1], 0)
    if zero != INT_MAX:
        err.append("WARNING: 0 coverage column %d (mincol=%d) found within alignment of %d seqs!\n"
                   % (zero, mincol, hdr.n))
        err.extend("row%u\n" % r for r in range(hdr.n))
        return 5, "".join(err) if rank == 0 else "", None
    own = range(lo, hi)
    cons_s, base, alpos = b"", {r: (int(lay.offset[r]), int(lay.numgaps[r]), lay.ofs[r]) for r in own}, []
    if mincol != INT_MAX:
        cons_s, edited = engine.refine_host(st, remove_gaps)
        base.update(edited)
        if remove_gaps:  # layout positions of the removed columns, in removal order
            cc = cons_cols.cpu().numpy() if hasattr(cons_cols, "cpu") else np.asarray(cons_cols)
            gaps = np.flatnonzero(cc[mincol:maxcol + 1] == ord("-")) + mincol
            alpos = (gaps - np.arange(gaps.size) + lay.minoffset).astype(np.int32)
    n_removed = len(alpos)
    # rows that change: all of them with removeConsGaps (removeClipGaps always moves ofs[0]),
    # else the clipped ones refineClipping may move
    fin = finish_rows(lay, [r for r in own if remove_gaps or (refine_clipping and (lay.clp5[r] or lay.clp3[r]))],
                      base, alpos, cons_s, mincol, remove_gaps, refine_clipping)
    if world > 1:
        # the exit code everywhere: a GError on any row ends the run (1); the rows only on rank 0
        bad_any = torch.tensor([1 if any(v[1] for v in fin.values()) else 0], dtype=torch.int64,
                               device=counts.device if dist.get_backend(group) == "nccl" else "cpu")
        dist.all_reduce(bad_any, op=dist.ReduceOp.MAX, group=group)
        fin = gather_rows(fin, group, counts.device)
        if rank != 0:
            return int(bad_any.item()), "", None
    for r in range(hdr.n):  # the per-row messages in row order, up to a row that GErrors
        if r in fin:
            err.append(fin[r][0])
            if fin[r][1]:
                return 1, "".join(err), None
    full = lay if world == 1 else Layout(layout_path, load=set(r for r in range(hdr.n) if r not in fin))
    counts_h = counts.cpu().numpy().astype("<i4")[: ncols * 6]
    out = [b"PWC1", struct.pack("<6i", ncols, lay.minoffset, -1 if mincol == INT_MAX else mincol, maxcol, len(cons_s),
                                n_removed), cons_s, counts_h.tobytes(), struct.pack("<I", hdr.n)]
    for r in range(hdr.n):
        if r in fin:
            _, _, off, ng, c5, c3, ofs = fin[r]
        else:
            off, ng, c5, c3, ofs = int(lay.offset[r]), int(lay.numgaps[r]), int(lay.clp5[r]), int(lay.clp3[r]), full.ofs[r]
        out.append(struct.pack("<4i", off, ng, c5, c3))
        out.append(np.asarray(ofs, dtype="<i2").tobytes())
    return 0, "".join(err), b"".join(out)
