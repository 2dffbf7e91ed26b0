"""pwasm_amd — MI355X-native pafreport hot path (gpertea/pwasm), Python side.

The product is native: libpwasm_amd.so (HIP kernels for gfx950 + C++ host pre-pass) and the
`pafreport` / `gapassem_consensus` executables built on it.  This module only binds the C-ABI
(include/pwasm_amd.h) with ctypes so bench.py and the tests can stage batches in device memory
owned by PyTorch and launch the kernels on PyTorch's stream.  There is no Python or CPU
implementation of the hot path here: if the library is missing every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import subprocess
import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
REPO = ROOT.parent
# PWASM_LIB selects another in-tree build of the same library (experiment builds, tools/exp_build.sh)
LIB_PATH = pathlib.Path(os.environ["PWASM_LIB"]) if os.environ.get("PWASM_LIB") else ROOT / "lib" / "libpwasm_amd.so"
CLI_PATH = ROOT / "bin" / "pafreport"
GA_CLI_PATH = ROOT / "bin" / "gapassem_consensus"

PW_OP_MATCH, PW_OP_SUB, PW_OP_INS, PW_OP_DEL = 0, 1, 2, 3
PW_CS_OK, PW_CS_PARSE, PW_CS_SPLICED, PW_CS_UNHANDLED, PW_CS_EMPTY, PW_CS_BOUNDS, PW_CS_NOSPACE = range(7)
PW_REC_OK, PW_REC_MISMATCH, PW_REC_MODSEQ = 0, 1, 2

DEV_PAD = 256  # readable bytes required past the end of the device query / literal arrays

# pafreport mode flags for pw_batch_from_files (same meaning as -G/-F/-C/-N)
FLAG_G, FLAG_F, FLAG_C, FLAG_N, FLAG_W = 1, 2, 4, 8, 16
FLAG_GPU_PACK = 32  # pw_batch_from_buffer: cs strings packed on the GPU by pw_runner_run (PW_BATCH_GPU_PACK)


class AlnDesc(ctypes.Structure):
    _fields_ = [("op_begin", ctypes.c_uint32), ("n_ops", ctypes.c_uint32), ("lit_begin", ctypes.c_uint32),
                ("ref", ctypes.c_uint32), ("offset", ctypes.c_int32), ("t_len", ctypes.c_int32),
                ("ev_begin", ctypes.c_uint64)]


class AlnResult(ctypes.Structure):
    _fields_ = [("text_off", ctypes.c_uint64), ("text_end", ctypes.c_uint64), ("page_first", ctypes.c_uint32),
                ("page_last", ctypes.c_uint32), ("text_len", ctypes.c_uint32), ("n_events", ctypes.c_uint32),
                ("err", ctypes.c_int32), ("err_a", ctypes.c_int32), ("err_b", ctypes.c_int32),
                ("err_c", ctypes.c_int32)]


class Page(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("len", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


PAGE_EVENTS, PAGE_BYTES = 64, 8192


def results_array(raw):
    """A results buffer (bytes / uint8 numpy / torch cpu tensor) as a numpy structured array."""
    import numpy as np
    dt = np.dtype([("text_off", "<u8"), ("text_end", "<u8"), ("page_first", "<u4"), ("page_last", "<u4"),
                   ("text_len", "<u4"), ("n_events", "<u4"), ("err", "<i4"), ("err_a", "<i4"), ("err_b", "<i4"),
                   ("err_c", "<i4")])
    assert dt.itemsize == ctypes.sizeof(AlnResult)
    a = np.asarray(raw).view(np.uint8).ravel()
    return a[: a.size - a.size % dt.itemsize].view(dt)


class ReportArgs(ctypes.Structure):
    _fields_ = [("desc", ctypes.c_void_p), ("ops", ctypes.c_void_p), ("lits", ctypes.c_void_p),
                ("qseq", ctypes.c_void_p), ("qoff", ctypes.c_void_p), ("qlen", ctypes.c_void_p),
                ("next_stop", ctypes.c_void_p), ("text", ctypes.c_void_p), ("results", ctypes.c_void_p),
                ("text_total", ctypes.c_uint64), ("n_alns", ctypes.c_uint32), ("skip_codan", ctypes.c_uint32),
                ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_uint64),
                ("n_ev_slots", ctypes.c_uint64), ("pages", ctypes.c_void_p), ("max_rec_ops", ctypes.c_uint32),
                ("n_short", ctypes.c_uint32), ("hot_pbits", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("n_queries", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class CsTotals(ctypes.Structure):
    _fields_ = [("q_total", ctypes.c_int32), ("t_total", ctypes.c_int32), ("n_ops", ctypes.c_uint32),
                ("n_lits", ctypes.c_uint32), ("n_events_max", ctypes.c_uint32), ("text_bound", ctypes.c_uint64)]


class BatchView(ctypes.Structure):
    _fields_ = [("desc", ctypes.c_void_p), ("ops", ctypes.c_void_p), ("lits", ctypes.c_void_p),
                ("qseq", ctypes.c_void_p), ("qoff", ctypes.c_void_p), ("qlen", ctypes.c_void_p),
                ("n_alns", ctypes.c_uint64), ("n_ops", ctypes.c_uint64), ("n_lits", ctypes.c_uint64),
                ("qseq_len", ctypes.c_uint64), ("n_queries", ctypes.c_uint64), ("text_total", ctypes.c_uint64),
                ("n_events_max", ctypes.c_uint64), ("alg_bytes_in", ctypes.c_uint64),
                ("skip_codan", ctypes.c_uint32)]


class MsaArgs(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_void_p), ("ofs", ctypes.c_void_p), ("row_off", ctypes.c_void_p),
                ("row_len", ctypes.c_void_p), ("col0", ctypes.c_void_p), ("clip_l", ctypes.c_void_p),
                ("clip_r", ctypes.c_void_p), ("slot_base", ctypes.c_void_p), ("scratch", ctypes.c_void_p),
                ("counts", ctypes.c_void_p), ("consensus", ctypes.c_void_p), ("minmax", ctypes.c_void_p),
                ("n_slots", ctypes.c_uint64), ("n_rows", ctypes.c_uint32), ("n_cols", ctypes.c_int32)]


class MsaRefineArgs(ctypes.Structure):
    _fields_ = [("gap_prefix", ctypes.c_void_p), ("tile_gaps", ctypes.c_void_p), ("cons_out", ctypes.c_void_p),
                ("cons_len", ctypes.c_void_p), ("row_offset", ctypes.c_void_p), ("ofs_out", ctypes.c_void_p),
                ("offset_out", ctypes.c_void_p), ("numgaps_out", ctypes.c_void_p), ("remove_gaps", ctypes.c_uint32),
                ("keep_clip_gaps", ctypes.c_uint32)]


class GaRow(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_void_p), ("ofs", ctypes.c_void_p), ("seqlen", ctypes.c_int32),
                ("offset", ctypes.c_int32), ("numgaps", ctypes.c_int32), ("clp5", ctypes.c_int32),
                ("clp3", ctypes.c_int32), ("revcompl", ctypes.c_int32), ("id", ctypes.c_char_p)]


# every function declared in include/pwasm_amd.h (tests check the export table against it)
_SIGS = {
    "pw_report_events": (ctypes.c_int, [ctypes.POINTER(ReportArgs), ctypes.c_void_p]),
    "pw_report_events_after": (ctypes.c_int, [ctypes.POINTER(ReportArgs), ctypes.c_void_p, ctypes.c_void_p]),
    "pw_stop_table_build": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    "pw_msa_slots": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    "pw_msa_scratch_words": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint32]),
    "pw_msa_columns": (ctypes.c_int, [ctypes.POINTER(MsaArgs), ctypes.c_void_p]),
    "pw_msa_count": (ctypes.c_int, [ctypes.POINTER(MsaArgs), ctypes.c_void_p]),
    "pw_msa_call": (ctypes.c_int, [ctypes.POINTER(MsaArgs), ctypes.c_void_p]),
    "pw_msa_call_cols": (ctypes.c_int, [ctypes.POINTER(MsaArgs), ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    "pw_msa_call_sharded": (ctypes.c_int, [ctypes.POINTER(MsaArgs), ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "pw_msa_refine_tiles": (ctypes.c_uint64, [ctypes.c_int32]),
    "pw_msa_refine": (ctypes.c_int, [ctypes.POINTER(MsaArgs), ctypes.POINTER(MsaRefineArgs), ctypes.c_void_p]),
    "pw_msa_columns_refine": (ctypes.c_int, [ctypes.POINTER(MsaArgs), ctypes.POINTER(MsaRefineArgs), ctypes.c_void_p]),
    "pw_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "pw_comm_init": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p, ctypes.c_int]),
    "pw_comm_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "pw_msa_counts_allreduce": (ctypes.c_int, [ctypes.POINTER(MsaArgs), ctypes.c_uint32, ctypes.c_void_p,
                                               ctypes.c_void_p]),
    "pw_msa_counts_reduce_scatter": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                    ctypes.c_void_p]),
    "pw_ga_row_remove_columns": (ctypes.c_int, [ctypes.POINTER(GaRow), ctypes.c_void_p, ctypes.c_uint64]),
    "pw_ga_row_finish": (ctypes.c_int, [ctypes.POINTER(GaRow), ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]),
    "pw_ga_rows_finish": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "pw_pack_cs_batch": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4),
    "pw_pack_cs": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t,
                                  ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(CsTotals),
                                  ctypes.POINTER(ctypes.c_int32)]),
    "pw_pafreport_main": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]),
    "pw_pafreport_main_exit": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]),  # (ends the process)
    "pw_batch_from_files": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                              ctypes.c_size_t]),
    "pw_batch_view_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(BatchView)]),
    "pw_batch_write_report": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_char_p]),
    "pw_report_page_count": (ctypes.c_uint64, [ctypes.c_uint64]),
    "pw_report_text_bytes": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
    "pw_report_workspace_bytes": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
    "pw_report_hot_pbits": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint64]),
    "pw_batch_write_items": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_char_p]),
    "pw_batch_free": (None, [ctypes.c_void_p]),
    "pw_batch_write_msa": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    "pw_version": (ctypes.c_char_p, []),
    "pw_gapassem_run": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32]),
    "pw_gapassem_run_ex": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                          ctypes.c_char_p, ctypes.c_char_p]),
    "pw_batch_from_files_shard": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                                                    ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]),
    "pw_items_merge": (ctypes.c_int, [ctypes.POINTER(ctypes.c_char_p), ctypes.c_uint32, ctypes.c_char_p,
                                      ctypes.c_char_p]),
    "pw_paf_split": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                       ctypes.c_char_p, ctypes.c_size_t]),
    "pw_split_lines": (ctypes.c_uint64, [ctypes.c_void_p]),
    "pw_split_bytes": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_uint32]),
    "pw_split_count": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_uint32]),
    "pw_split_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "pw_split_free": (None, [ctypes.c_void_p]),
    "pw_batch_from_buffer": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                               ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_char_p,
                                               ctypes.c_size_t]),
    "pw_batch_item_count": (ctypes.c_uint64, [ctypes.c_void_p]),
    "pw_batch_items": (ctypes.c_int, [ctypes.c_void_p] * 8 + [ctypes.POINTER(ctypes.c_uint64)]),
    "pw_batch_write_at": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                                                 ctypes.c_void_p, ctypes.c_uint64]),
    "pw_batch_write_range": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                                                    ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]),
    "pw_batch_render_range": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                                                     ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]),
    "pw_gather_write": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint64]),
    "pw_batch_cuts": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_uint64]),
    "pw_batch_genomes": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "pw_batch_genomes_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "pw_genome_table": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    "pw_runner_create": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]),
    "pw_runner_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.POINTER(ctypes.c_uint64)]),
    "pw_runner_fetch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                       ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]),
    "pw_runner_genome_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_void_p]),
    "pw_runner_free": (None, [ctypes.c_void_p]),
}

_lib = None


def build(jobs: int = 8) -> None:
    """Compile the HIP library, CLIs, oracle and synth tool in-tree (make)."""
    subprocess.run(["make", f"-j{jobs}"], cwd=str(REPO), check=True)


def lib() -> ctypes.CDLL:
    """The native library; raises if it was not built (there is no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"pwasm_amd: native library missing ({LIB_PATH}); run `make` / __graft_entry__.build()")
        L = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in _SIGS.items():
            if os.environ.get("PWASM_LIB") and not hasattr(L, name):
                continue  # (an older experiment build: tools/exp_build.py)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def pack_cs(cs: str, offset: int, qlen: int):
    """CPU pre-pass on one cs string -> (rc, ops list, literal bytes, totals, err_pos)."""
    L = lib()
    n = len(cs) + 1
    ops = (ctypes.c_uint32 * n)()
    lits = (ctypes.c_uint8 * n)()
    tot = CsTotals()
    epos = ctypes.c_int32(0)
    rc = L.pw_pack_cs(cs.encode(), offset, qlen, ops, n, lits, n, ctypes.byref(tot), ctypes.byref(epos))
    return rc, list(ops[:tot.n_ops]), bytes(lits[:tot.n_lits]), tot, epos.value


CS_REC = np.dtype([("q_total", "<i4"), ("t_total", "<i4"), ("n_ops", "<u4"), ("n_lits", "<u4"),
                   ("n_events_max", "<u4"), ("flags", "<u4"), ("text_bound", "<u8")])
PACK_HOST, PACK_ACGT = 1, 2
REPORT_BUILD_NEXT_STOP = 1  # pw_report_args.flags


def pack_cs_gpu(cs_list, offsets, qlens, device: str = "cuda:0"):
    """pw_pack_cs_batch on the GPU for a list of cs strings (bytes) -> (ops uint32[], lits
    uint8[], cs_off uint64[n+1], records CS_REC[n]); record i's ops / literal bytes start at
    cs_off[i] (PACK_HOST records: pack them with pack_cs)."""
    import torch
    n = len(cs_list)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(c) for c in cs_list], dtype=np.uint64)
    text = np.frombuffer(b"".join(cs_list) + b"\0" * 16, dtype=np.uint8)
    t = lambda a: torch.from_numpy(np.array(a, copy=True)).to(device)
    d_text, d_off = t(text), t(off.view(np.int64))
    d_o, d_q = t(np.asarray(offsets, dtype=np.int32)), t(np.asarray(qlens, dtype=np.int32))
    tot = int(off[-1]) + 16
    d_ops = torch.zeros(tot, dtype=torch.int32, device=device)
    d_lits = torch.zeros(tot, dtype=torch.uint8, device=device)
    d_rec = torch.zeros(max(n, 1) * CS_REC.itemsize, dtype=torch.uint8, device=device)
    rc = lib().pw_pack_cs_batch(d_text.data_ptr(), d_off.data_ptr(), d_o.data_ptr(), d_q.data_ptr(), n,
                                d_ops.data_ptr(), d_lits.data_ptr(), d_rec.data_ptr(),
                                torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError(f"pw_pack_cs_batch: {rc}")
    torch.cuda.synchronize()
    recs = d_rec.cpu().numpy().view(CS_REC)[:n]
    return d_ops.cpu().numpy().view(np.uint32), d_lits.cpu().numpy(), off, recs


def paf_split(paf: str, lo: int, hi: int, nshards: int):
    """pw_paf_split: the lines starting in bytes [lo, hi) of the PAF routed to their target-genome
    shards -> (lines in the range, [bytes uint8 per owner], [index in the range uint32 per owner])."""
    L = lib()
    err = ctypes.create_string_buffer(4096)
    h = L.pw_paf_split(str(paf).encode(), lo, hi, nshards, err, 4096)
    if not h:
        raise RuntimeError("pw_paf_split: " + err.value.decode(errors="replace"))
    try:
        n = int(L.pw_split_lines(h))
        data, idx = [], []
        for o in range(nshards):
            b = np.empty(int(L.pw_split_bytes(h, o)), dtype=np.uint8)
            i = np.empty(int(L.pw_split_count(h, o)), dtype=np.uint32)
            if L.pw_split_get(h, o, b.ctypes.data, i.ctypes.data) != 0:
                raise RuntimeError("pw_split_get failed")
            data.append(b)
            idx.append(i)
        return n, data, idx
    finally:
        L.pw_split_free(h)


class HostBatch:
    """A PAF batch packed by the C++ pre-pass (pw_batch_from_files), arrays viewable as numpy."""

    def __init__(self, fasta: str, paf: str = None, flags: int = 0, shard: int = 0, nshards: int = 1, _handle=None):
        """shard / nshards: pack only this rank's lines (target-name hash, pw_batch_from_files_shard)."""
        L = lib()
        if _handle is None:
            err = ctypes.create_string_buffer(4096)
            h = L.pw_batch_from_files_shard(fasta.encode(), paf.encode(), flags, shard, nshards, err, 4096)
            if not h:
                raise RuntimeError("pw_batch_from_files: " + err.value.decode(errors="replace"))
        else:
            h = _handle
        self._h = h
        self.view = BatchView()
        if L.pw_batch_view_get(h, ctypes.byref(self.view)) != 0:
            raise RuntimeError("pw_batch_view_get failed")

    @classmethod
    def from_buffer(cls, fasta: str, text, line_no, flags: int = 0, prev=None):
        """pw_batch_from_buffer: lines ended by '\\n' in `text` (uint8 array) with their global input
        lines `line_no` (uint64, ascending); prev = the batch of the lines before (its q~t dedupe
        state moves over)."""
        L = lib()
        text = np.ascontiguousarray(text, dtype=np.uint8)
        line_no = np.ascontiguousarray(line_no, dtype=np.uint64)
        err = ctypes.create_string_buffer(4096)
        h = L.pw_batch_from_buffer(fasta.encode(), text.ctypes.data if text.size else None, text.size,
                                   line_no.ctypes.data if line_no.size else None, line_no.size, flags,
                                   prev._h if prev is not None else None, err, 4096)
        if not h:
            raise RuntimeError("pw_batch_from_buffer: " + err.value.decode(errors="replace"))
        return cls(fasta, _handle=h)

    def items(self, text_host, results_host, pages_host):
        """Output items (global line, status, stdout bytes, stderr bytes) up to the first that ends
        the run (pw_batch_items)."""
        L = lib()
        n = int(L.pw_batch_item_count(self._h))
        line = np.zeros(max(n, 1), dtype=np.uint64)
        st = np.zeros(max(n, 1), dtype=np.int32)
        on = np.zeros(max(n, 1), dtype=np.uint64)
        en = np.zeros(max(n, 1), dtype=np.uint64)
        k = ctypes.c_uint64(0)
        rc = L.pw_batch_items(self._h, text_host.ctypes.data, results_host.ctypes.data, pages_host.ctypes.data,
                              line.ctypes.data, st.ctypes.data, on.ctypes.data, en.ctypes.data, ctypes.byref(k))
        if rc != 0:
            raise RuntimeError(f"pw_batch_items: {rc}")
        k = int(k.value)
        return line[:k], st[:k], on[:k], en[:k]

    def write_at(self, text_host, results_host, pages_host, fd: int, out_off, err_bytes: int) -> bytes:
        """pw_batch_write_at: stdout of the first len(out_off) items pwritten at out_off into fd; returns
        their stderr bytes."""
        out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
        eb = ctypes.create_string_buffer(max(int(err_bytes), 1))
        rc = lib().pw_batch_write_at(self._h, text_host.ctypes.data, results_host.ctypes.data, pages_host.ctypes.data,
                                     fd, out_off.ctypes.data if out_off.size else None, out_off.size, eb,
                                     int(err_bytes))
        if rc != 0:
            raise RuntimeError(f"pw_batch_write_at: {rc}")
        return eb.raw[: int(err_bytes)]

    def write_range(self, text_host, results_host, pages_host, fd: int, first: int, out_off, err_bytes: int) -> bytes:
        """pw_batch_write_range: stdout of items [first, first + len(out_off)) pwritten at out_off into
        fd; returns their stderr bytes."""
        out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
        eb = ctypes.create_string_buffer(max(int(err_bytes), 1))
        rc = lib().pw_batch_write_range(self._h, text_host.ctypes.data, results_host.ctypes.data,
                                        pages_host.ctypes.data, fd, int(first),
                                        out_off.ctypes.data if out_off.size else None, out_off.size, eb,
                                        int(err_bytes))
        if rc != 0:
            raise RuntimeError(f"pw_batch_write_range: {rc}")
        return eb.raw[: int(err_bytes)]

    def render_range(self, text_host, results_host, pages_host, first: int, out_bytes: int, n_items: int,
                     err_bytes: int, out=None):
        """pw_batch_render_range: (stdout bytes of items [first, first + n_items) back to back as a
        uint8 array of out_bytes, their stderr bytes).  out: a contiguous uint8 array of at least
        out_bytes to render into (e.g. a slice of a reused send buffer)."""
        if out is None:
            out = np.empty(max(int(out_bytes), 1), dtype=np.uint8)
        elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < int(out_bytes):
            raise ValueError("render_range: out must be a contiguous uint8 array of at least out_bytes")
        elif out.size == 0:
            out = np.empty(1, dtype=np.uint8)
        eb = ctypes.create_string_buffer(max(int(err_bytes), 1))
        rc = lib().pw_batch_render_range(self._h, text_host.ctypes.data, results_host.ctypes.data,
                                         pages_host.ctypes.data, int(first), int(n_items), out.ctypes.data,
                                         int(out_bytes), eb, int(err_bytes))
        if rc != 0:
            raise RuntimeError(f"pw_batch_render_range: {rc}")
        return out[: int(out_bytes)], eb.raw[: int(err_bytes)]

    def array(self, name: str):
        import numpy as np
        v = self.view
        spec = {"desc": (v.desc, v.n_alns * ctypes.sizeof(AlnDesc), np.uint8),
                "ops": (v.ops, v.n_ops, np.uint32), "lits": (v.lits, v.n_lits, np.uint8),
                "qseq": (v.qseq, v.qseq_len, np.uint8), "qoff": (v.qoff, v.n_queries, np.uint64),
                "qlen": (v.qlen, v.n_queries, np.int32)}[name]
        ptr, n, dt = spec
        if n == 0:
            return np.zeros(0, dtype=dt)
        ct = np.ctypeslib.as_ctypes_type(dt)
        buf = (ct * int(n)).from_address(int(ptr))
        return np.ctypeslib.as_array(buf).copy()

    def max_rec_ops(self) -> int:
        """Largest op count of a record (pw_report_args.max_rec_ops)."""
        if getattr(self, "_max_ops", None) is None:
            d = self.array("desc").view(np.uint32).reshape(-1, 8)
            self._max_ops = int(d[:, 1].max()) if d.size else 0
            self._n_short = int((d[:, 1] <= 64).sum()) if d.size else 0
        return self._max_ops

    def n_short(self) -> int:
        """Records of at most 64 ops (pw_report_args.n_short)."""
        self.max_rec_ops()
        return self._n_short

    def write_report(self, text_host, results_host, pages_host, path: str) -> int:
        """Headers + event text for a finished batch (numpy arrays on the host)."""
        return lib().pw_batch_write_report(self._h, text_host.ctypes.data, results_host.ctypes.data,
                                           pages_host.ctypes.data, path.encode())

    def write_items(self, text_host, results_host, pages_host, path: str) -> int:
        """The same output cut into line-tagged items (PWI1) for the multi-GPU shard merge."""
        return lib().pw_batch_write_items(self._h, text_host.ctypes.data, results_host.ctypes.data,
                                          pages_host.ctypes.data, path.encode())

    def write_report_from(self, dev: dict, path: str) -> int:
        """write_report with the device buffers of stage_batch() copied to the host."""
        return self.write_report(dev["text"].cpu().numpy(), dev["results"].cpu().numpy(), dev["pages"].cpu().numpy(),
                                 path)

    def write_items_from(self, dev: dict, path: str) -> int:
        return self.write_items(dev["text"].cpu().numpy(), dev["results"].cpu().numpy(), dev["pages"].cpu().numpy(),
                                path)

    def write_msa(self, path: str) -> int:
        """-w: the MSA of the last query run as multi-FASTA (needs FLAG_W)."""
        return lib().pw_batch_write_msa(self._h, str(path).encode())

    def genomes(self):
        """-> (genome index per record [n_alns] uint32, aligned target bases [n_alns] int32,
        target names) for the per-genome tables."""
        import numpy as np
        L = lib()
        nb = ctypes.c_uint64(0)
        ng = int(L.pw_batch_genomes(self._h, ctypes.byref(nb)))
        n = int(self.view.n_alns)
        gof = np.zeros(max(n, 1), dtype=np.uint32)
        taln = np.zeros(max(n, 1), dtype=np.int32)
        names = ctypes.create_string_buffer(max(int(nb.value), 1))
        if L.pw_batch_genomes_get(self._h, gof.ctypes.data, taln.ctypes.data, names) != 0:
            raise RuntimeError("pw_batch_genomes_get failed")
        nm = names.raw[: int(nb.value)].split(b"\0")[:ng]
        return gof[:n], taln[:n], nm

    def close(self):
        if self._h:
            lib().pw_batch_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _env_flag(name):
    """An integer switch read as the C host reads it (atoi(getenv(name)) != 0): unset, empty, "0"
    or a non-number are off."""
    import re
    m = re.match(r"\s*[+-]?\d+", os.environ.get(name, ""))
    return m is not None and int(m.group(0)) != 0


def report_args(batch: HostBatch, dev: dict) -> ReportArgs:
    """pw_report_args over the device tensors of stage_batch()."""
    v = batch.view
    a = ReportArgs()
    a.desc = dev["desc"].data_ptr()
    a.ops = dev["ops"].data_ptr()
    a.lits = dev["lits"].data_ptr()
    a.qseq = dev["qseq"].data_ptr()
    a.qoff = dev["qoff"].data_ptr()
    a.qlen = dev["qlen"].data_ptr()
    a.next_stop = 0 if v.skip_codan else dev["next_stop"].data_ptr()
    a.text = dev["text"].data_ptr()
    a.results = dev["results"].data_ptr()
    a.text_total = dev["text"].numel()
    a.n_alns = int(v.n_alns)
    a.skip_codan = int(v.skip_codan)
    a.workspace = dev["work"].data_ptr()
    a.workspace_bytes = dev["work"].numel()
    a.n_ev_slots = int(v.n_events_max)
    a.pages = dev["pages"].data_ptr()
    a.max_rec_ops = batch.max_rec_ops()
    a.n_short = 0 if _env_flag("PW_NO_PAIRS") else batch.n_short()
    # 16-byte event records when the query positions / indices fit (PW_HOT32=1: 32-byte ones)
    ql = batch.array("qlen")
    a.hot_pbits = 0 if _env_flag("PW_HOT32") else int(lib().pw_report_hot_pbits(int(ql.max()) if ql.size else 0,
                                                                               int(v.n_queries)))
    a.n_queries = int(v.n_queries)
    return a


def run_report(batch: HostBatch, dev: dict, stream_ptr: int) -> None:
    """pw_report_events on device tensors in `dev`, the next-stop table built by the pass itself
    (PW_REPORT_BUILD_NEXT_STOP; unless -F/-N) — or, with PW_NS_SEPARATE=1, by pw_stop_table_build
    launched before it."""
    L = lib()
    v = batch.view
    a = report_args(batch, dev)
    if not v.skip_codan:
        if _env_flag("PW_NS_SEPARATE"):
            rc = L.pw_stop_table_build(dev["qseq"].data_ptr(), dev["qoff"].data_ptr(), dev["qlen"].data_ptr(),
                                       int(v.n_queries), dev["next_stop"].data_ptr(), stream_ptr)
            if rc != 0:
                raise RuntimeError(f"pw_stop_table_build: {rc}")
        else:
            a.flags |= REPORT_BUILD_NEXT_STOP
    rc = L.pw_report_events(ctypes.byref(a), stream_ptr)
    if rc != 0:
        raise RuntimeError(f"pw_report_events: {rc}")


def fetch_outputs(dev: dict, alloc=None):
    """Host copies of a finished pass: (text up to its last used byte, results, pages) as numpy.
    alloc(n) -> a host uint8 tensor of n bytes to copy the text into (a reused pinned buffer: no
    page faults on the copy, no unmap when the batch is dropped); None: a fresh pageable array."""
    res = dev["results"].cpu().numpy()
    pages = dev["pages"].cpu().numpy()
    pg = pages.view(np.uint8)[: pages.size - pages.size % 16].view(np.dtype([("off", "<u8"), ("len", "<u4"),
                                                                              ("pad", "<u4")]))
    used = max(int((pg["off"] + pg["len"]).max()) if pg.size else 0, 1)
    if alloc is None:
        return dev["text"][:used].cpu().numpy(), res, pages
    dst = alloc(used)
    dst.copy_(dev["text"][:used])
    return dst.numpy(), res, pages


def stage_batch(batch: HostBatch, device: str = "cuda:0") -> dict:
    """Copy a packed batch into device tensors (inputs resident in HBM) + output buffers."""
    import numpy as np
    import torch
    v = batch.view
    dev = {}
    for name in ("desc", "ops", "lits", "qseq", "qoff", "qlen"):
        arr = batch.array(name)
        if arr.size == 0:
            arr = np.zeros(1, dtype=arr.dtype)
        if arr.dtype == np.uint64:  # torch only needs the bytes
            arr = arr.view(np.uint8)
        if name in ("lits", "qseq"):  # the kernel reads up to 256 bytes past the end (16-byte staging loads)
            arr = np.concatenate([arr, np.zeros(DEV_PAD, dtype=arr.dtype)])
        dev[name] = torch.from_numpy(arr).to(device)
    dev["next_stop"] = torch.empty(max(int(v.qseq_len), 1), dtype=torch.int32, device=device)
    L = lib()
    dev["text"] = torch.empty(max(int(L.pw_report_text_bytes(int(v.n_events_max), int(v.text_total))), 16),
                              dtype=torch.uint8, device=device)
    dev["pages"] = torch.zeros(max(int(L.pw_report_page_count(int(v.n_events_max))), 1) * ctypes.sizeof(Page),
                               dtype=torch.uint8, device=device)
    dev["work"] = torch.empty(int(lib().pw_report_workspace_bytes(int(v.n_events_max), int(v.n_alns))), dtype=torch.uint8,
                              device=device)
    dev["results"] = torch.empty(max(int(v.n_alns), 1) * ctypes.sizeof(AlnResult), dtype=torch.uint8,
                                 device=device)
    return dev


def gather_write(fd: int, file_off: int, src, src_off, lens) -> None:
    """pw_gather_write: spans src[src_off[k], + lens[k]) in order, written contiguously at file_off."""
    src_off = np.ascontiguousarray(src_off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    rc = lib().pw_gather_write(int(fd), int(file_off), src.ctypes.data if src.size else None,
                               src_off.ctypes.data if src_off.size else None, lens.ctypes.data if lens.size else None,
                               int(lens.size))
    if rc != 0:
        raise RuntimeError(f"pw_gather_write: {rc}")


def items_merge(paths, out_path=None, err_path=None) -> int:
    """pw_items_merge: the merged stdout / stderr of all shards' item streams; returns the exit code."""
    arr = (ctypes.c_char_p * len(paths))(*[str(p).encode() for p in paths])
    return lib().pw_items_merge(arr, len(paths), str(out_path).encode() if out_path else None,
                                str(err_path).encode() if err_path else None)


GENOME_ROW = 16  # sizeof(pw_genome_row)


class Runner:
    """pw_runner: the CLI's device session for the batches of one query set (queries and the
    next-stop table uploaded once on the current device; device buffers reused; cs strings of
    FLAG_GPU_PACK batches packed on the GPU).  run(batch) -> (pages, text bytes); fetch(text, ...)
    -> (text, results, pages) as numpy, the text copied into `text` (a host uint8 tensor / array
    of at least that many bytes, e.g. a pinned buffer)."""

    def __init__(self, batch: HostBatch):
        err = ctypes.create_string_buffer(512)
        self._h = lib().pw_runner_create(batch._h, err, len(err))
        if not self._h:
            raise RuntimeError("pw_runner_create: " + err.value.decode(errors="replace"))
        self._n = 0

    def run(self, batch: HostBatch):
        npg, used = ctypes.c_uint64(0), ctypes.c_uint64(0)
        rc = lib().pw_runner_run(self._h, batch._h, ctypes.byref(npg), ctypes.byref(used))
        if rc != 0:
            raise RuntimeError(f"pw_runner_run: {rc}")
        self._n = int(batch.view.n_alns)
        return int(npg.value), int(used.value)

    def fetch(self, text, n_pages: int, used: int):
        res = np.empty(max(self._n, 1) * ctypes.sizeof(AlnResult), np.uint8)
        pages = np.empty(max(n_pages, 1) * ctypes.sizeof(Page), np.uint8)
        tp = text.data_ptr() if hasattr(text, "data_ptr") else text.ctypes.data
        cap = text.numel() if hasattr(text, "numel") else text.size
        rc = lib().pw_runner_fetch(self._h, res.ctypes.data, self._n, pages.ctypes.data, n_pages, tp if used else None,
                                   cap)
        if rc != 0:
            raise RuntimeError(f"pw_runner_fetch: {rc}")
        t = text.numpy() if hasattr(text, "numpy") else text
        return t[:max(used, 1)], res, pages

    def genome_rows(self, batch: HostBatch):
        """(rows as uint8 [n_genomes * 16], target names) of the last run batch."""
        gof, taln, names = batch.genomes()
        rows = np.zeros(max(len(names), 1) * GENOME_ROW, np.uint8)
        n = int(batch.view.n_alns)
        rc = lib().pw_runner_genome_rows(self._h, np.ascontiguousarray(gof, np.uint32).ctypes.data if n else None,
                                         np.ascontiguousarray(taln, np.int32).ctypes.data if n else None, n, len(names),
                                         rows.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"pw_runner_genome_rows: {rc}")
        return rows[: len(names) * GENOME_ROW], names

    def close(self):
        if self._h:
            lib().pw_runner_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def version() -> str:
    return lib().pw_version().decode()
