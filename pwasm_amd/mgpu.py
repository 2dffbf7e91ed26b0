"""Multi-GPU `pafreport`: one process per GPU, launched by torchrun.

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m pwasm_amd.mgpu [-G|-F] [-C|-N] -r cds.fa mappings.paf [-o report.txt] [--genome-table t.tsv]

Replaces the reference's sequential record loop (pafreport.cpp:303-436) over a node:

  every rank    packs ONLY the PAF lines of its target-genome shard (crc32 of PAF column 6 mod
                world; pw_batch_from_files_shard, multi-threaded host pre-pass) — gene mode's
                first-occurrence q~t dedupe (pafreport.cpp:319-334) is keyed by the target, so it
                is shard-local — stages them in its GPU's HBM and runs the HIP pass
                (pw_stop_table_build + pw_report_events);
  per-genome    pw_genome_table sums each target's alignments / event lines / aligned bases on the
  tables        device; the rows and target names of all ranks are all-gathered (RCCL over xGMI
                with the "nccl" backend) so rank 0 holds the node-wide table (--genome-table);
  items         every rank writes its report as line-tagged items (PWI1, pw_batch_write_items);
                rank 0 merges them by global input line (pw_items_merge) into exactly the stdout /
                stderr / exit code of a single-process run.
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


def main(argv=None) -> int:
    import torch
    import torch.distributed as dist

    import pwasm_amd as pw

    argv = sys.argv[1:] if argv is None else argv
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("PW_DIST_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend=backend)
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
    # a shared scratch directory for the item streams (one node)
    if world > 1:
        obj = [extra.get("tmpdir") or (tempfile.mkdtemp(prefix="pwmg_") if rank == 0 else None)]
        dist.broadcast_object_list(obj, src=0)
        tmp = obj[0]
    else:
        tmp = extra.get("tmpdir") or tempfile.mkdtemp(prefix="pwmg_")
    os.makedirs(tmp, exist_ok=True)
    err = None
    try:
        b = pw.HostBatch(fa, nonopt[0], flags, rank, world)
    except RuntimeError as e:
        err = str(e)
    if world > 1:
        errs = [None] * world
        dist.all_gather_object(errs, err)
        err = next((e for e in errs if e), None)
    if err:
        if rank == 0:
            sys.stderr.write(err.split(": ", 1)[-1] if err.startswith("pw_batch_from_files") else err)
        return 1
    stream = torch.cuda.current_stream()
    dev = pw.stage_batch(b, device)
    pw.run_report(b, dev, stream.cuda_stream)
    rows, names, gt = genome_rows(b, dev, stream.cuda_stream)
    launch_genome_table(dev, rows, gt, stream.cuda_stream)
    items = os.path.join(tmp, f"items{rank}.pwi")
    rc = b.write_items_from(dev, items)
    if rc != 0:
        raise RuntimeError(f"pw_batch_write_items: {rc}")
    want_table = "genome-table" in extra
    if world > 1:
        all_rows = [x.cpu().numpy() for x in gather_ragged(rows)]
        nb = b"\0".join(names)
        nt = torch.from_numpy(np.frombuffer(nb, dtype=np.uint8).copy() if nb else np.zeros(0, np.uint8)).to(device)
        all_names = [bytes(x.cpu().numpy()).split(b"\0") if x.numel() else [] for x in gather_ragged(nt)]
        dist.barrier()
    else:
        torch.cuda.synchronize()
        all_rows, all_names = [rows.cpu().numpy()], [names]
    code = 0
    if rank == 0:
        code = pw.items_merge([os.path.join(tmp, f"items{r}.pwi") for r in range(world)], opts.get("o") or None)
        if want_table:
            write_genome_table(extra["genome-table"], all_rows, all_names)
    if world > 1:
        c = torch.tensor([code], dtype=torch.int64, device=device)
        if dist.get_backend() == "gloo":
            c = c.cpu()
        dist.broadcast(c, src=0)
        code = int(c.item())
        dist.barrier()
    if rank == 0 and not extra.get("tmpdir"):
        for r in range(world):
            try:
                os.remove(os.path.join(tmp, f"items{r}.pwi"))
            except OSError:
                pass
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
