#!/usr/bin/env python3
"""bench.py — pafreport hot path on MI355X: cs-events classified per second.

A "step" = one pass of the hot path over one batch already resident in HBM: the next-stop
table build (by the pass's first kernel beside the decode: PW_REPORT_BUILD_NEXT_STOP) + the
decode/classify/codon/render kernels (pw_report_events_after) over every record of the batch.  At N=1 the batch is BASELINE.json
configs[1] (cfg2: 100k synthetic minimap2-style records, 1,000 CDS of 1-5 kb, ~1% ONT-style
errors, run with -G -C).  With N>1 every rank processes its own cfg2-sized shard (different
seed = different target genomes; weak scaling, no data-path collective; the per-genome tables
are all-gathered over RCCL every step); the timed region is bracketed by barrier + synchronize,
the max over ranks is reported.  Beside it at every N, N = 1 included (sub-object "cfg3", and its
strong-scaling figures as the top-level "scaling_cfg3"): BASELINE configs[2], the one 10M-record
set sharded by target genome over the N ranks, and the node's end-to-end run of it
(pwasm_amd.mgpu) — speedup(N) = scaling_cfg3.value(N) / scaling_cfg3.value(1).

`python3 bench.py --gpus N` with no WORLD_SIZE in the environment launches the N ranks itself
(one process per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set
as torchrun sets them) before anything touches the GPU; under torchrun WORLD_SIZE must equal
--gpus.

Also reported (rank 0): roofline of the dominant kernel sequence (algorithmic bytes / the pass's
average GPU time — HIP events around the K timed passes, divided by K — vs 8 TB/s) and the CPU
baseline: the single-threaded oracle restatement
(oracle/pafreport_oracle, kind "port") on a bounded sample of the same workload, 1 core.
"""
import argparse
import filecmp
import json
import os
import pathlib
import shutil
import subprocess
import sys
import tempfile
import time

REPO = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=None,
                    help="2 (default at N=1: BASELINE configs[1]); 3 (default at N>1: the 10M-record set sharded "
                         "by target genome, configs[2]); 5 (GapAssem, configs[4])")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="records timed on the CPU oracle (default: the whole cfg2 batch; 100k records of cfg3, "
                         "10 of cfg4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle diff + end-to-end CLI run")
    ap.add_argument("--remove-gaps", action="store_true", help="cfg5: MSAColumns::removeConsGaps=true")
    ap.add_argument("--no-e2e", action="store_true", help="cfg3: skip the end-to-end pwasm_amd.mgpu leg")
    ap.add_argument("--no-gapassem", action="store_true", help="N = 1, cfg2: skip the cfg5 (GapAssem) sub-object")
    ap.add_argument("--e2e-parity", action="store_true", help="N > 1: CRC the end-to-end report against the oracle")
    ap.add_argument("--no-cfg3", action="store_true", help="skip the cfg3 (10M records sharded) sub-object")
    ap.add_argument("--cfg3-scale", type=float, default=1.0, help="scale of the cfg3 sub-object's record set")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC-derived HBM bytes per pass (profiles/run_prof.sh summary of the same command)")
    args = ap.parse_args()
    plan = launch_plan(args.gpus, sys.argv[1:], os.environ)
    if isinstance(plan, str):
        log(f"bench.py: {plan}")
        sys.exit(2)
    if plan:  # python3 bench.py --gpus N: start the N ranks (nothing here has touched torch / HIP)
        sys.exit(run_ranks(plan))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank_thread_share()
    if args.config is None:
        args.config = 2
    if args.traffic_json is None:  # the newest committed profile of the same command (profiles/run_prof.sh)
        args.traffic_json = latest_profile(args.config)

    import numpy as np
    import torch
    import torch.distributed as dist

    import pwasm_amd as pw

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:  # PW_DIST_BACKEND=gloo: rehearsal with several ranks on one GPU (RCCL refuses that)
        # (c10d / gloo announce their connections on fd 1: keep stdout to the one JSON line)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend=os.environ.get("PW_DIST_BACKEND",
                                                           "nccl" if torch.cuda.is_available() else "gloo"))
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    local = local % max(torch.cuda.device_count(), 1)
    dev_name = f"cuda:{local}"
    torch.cuda.set_device(local)
    if args.config == 5:
        out = bench_gapassem(args, world, rank, dev_name)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    out = report_leg(args, args.config, world, rank, dev_name)
    subs = sub_objects(world, args)
    if "cfg3" in subs:
        # BASELINE configs[2] beside the cfg2 line, at EVERY N (N = 1 included, so the driver's 1 -> 8
        # run has the denominator of the north star's scaling target): the one 10M-record set sharded
        # by target genome over the N ranks (strong scaling) + the node's end-to-end run of it
        torch.cuda.empty_cache()
        c3 = argparse.Namespace(**{**vars(args), "scale": args.cfg3_scale, "traffic_json": None, "no_parity": True,
                                   "no_cpu_baseline": True})
        sub = report_leg(c3, 3, world, rank, dev_name)
        if rank == 0:
            out["cfg3"] = {k: sub[k] for k in CFG3_KEYS}
            out["scaling_cfg3"] = scaling_cfg3(sub, world)
    if rank == 0:
        out["config"]["ranks"] = world
        out["config"]["backend"] = dist.get_backend() if dist.is_initialized() else "none"
        out["config"]["launcher"] = os.environ.get("PW_BENCH_LAUNCHER", "torchrun" if world > 1 else "single process")
        if "gapassem" in subs:
            # BASELINE configs[4] beside it, timed in its own region after the cfg2 one (cfg2's
            # device buffers released first): the GapAssem step, its roofline, parity, CPU baseline
            torch.cuda.empty_cache()
            ga = argparse.Namespace(**{**vars(args), "config": 5, "scale": 1.0, "remove_gaps": False,
                                       "traffic_json": latest_profile(5)})
            g = bench_gapassem(ga, 1, 0, dev_name)
            out["gapassem"] = {k: g[k] for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "dtype",
                                                 "config", "parity", "roofline", "cpu_baseline")}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


CFG3_KEYS = ("value", "unit", "n_gpus", "steps", "ms_per_step", "scaling", "config", "roofline", "e2e")


def sub_objects(world, args):
    """The sub-objects the bench line carries beside its own leg (pure; tests/test_bench_launch.py):
    "cfg3" (BASELINE configs[2], the 10M-record set sharded over the N ranks) at every N when the
    line is cfg2, "gapassem" (configs[4]) at N = 1."""
    subs = []
    if args.config == 2 and not args.no_cfg3:
        subs.append("cfg3")
    if world == 1 and args.config == 2 and not args.no_gapassem:
        subs.append("gapassem")
    return subs


def scaling_cfg3(sub, world):
    """Where a scaling reader looks: the strong-scaling figures of the one cfg3 set at this N.  The
    speedup at N is read from two bench lines of the same command, speedup(N) = value(N) / value(1)
    (kernel pass over the node, events/s) and e2e_wall_s(1) / e2e_wall_s(N) (PAF text to report
    file through pwasm_amd.mgpu); north_star's target is >= 6 at N = 8."""
    e2e = sub.get("e2e") or {}
    return {"value": sub["value"], "unit": sub["unit"], "n_gpus": world, "scaling": "strong",
            "records": sub["config"].get("records_total"), "events": sub["config"].get("events_total"),
            "kernel_ms_per_pass": sub["roofline"]["kernel_ms"], "ms_per_step": sub["ms_per_step"],
            "e2e_wall_s": e2e.get("wall_s"), "e2e_events_per_s": e2e.get("events_per_s"),
            "speedup_formula": "value(N) / value(1); e2e: e2e_wall_s(1) / e2e_wall_s(N); same cfg3 set, same scale"}


def report_leg(args, config, world, rank, dev_name):
    """One pafreport pass benchmark (config 2 weak / 3 sharded by target genome); the JSON object
    on rank 0, None elsewhere."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import pwasm_amd as pw

    # ---- data (synthetic, seeded; generated outside the timed region).  cfg3 is ONE 10M-record
    # set: rank r generates exactly the lines of its target-genome shard (crc32(target) % N == r,
    # the rule of pw_batch_from_files_shard / pwasm_amd.mgpu) — strong scaling.  Other configs
    # at N > 1: one independent batch per rank (weak scaling).
    sharded = config == 3
    tmp = tempfile.mkdtemp(prefix=f"pwbench{rank}_")
    if sharded and world > 1:  # one 10M-record file for the node (rank 0 writes it; ranks share it)
        box = [tmp if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        shared = box[0]
    else:
        shared = tmp
    fa, paf = os.path.join(shared, "q.fa"), os.path.join(shared, "a.paf")
    seed = 3 if sharded else (2 + 1000 * rank if config == 2 else config + 1000 * rank)
    t0 = time.time()
    cmd = [str(REPO / "synth/build/pwsynth"), "paf", "--config", str(config), "--scale", str(args.scale),
           "--seed", str(seed), "--fa", fa, "--paf", paf]
    if config in (3, 4):
        cmd += ["--threads", str(host_threads())]
    if not (sharded and world > 1 and rank != 0):
        subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    if sharded and world > 1:
        dist.barrier()
    t_gen = time.time() - t0
    flags = pw.FLAG_G | pw.FLAG_C if config in (1, 2, 3) else 0
    # cfg3 over N ranks: rank r packs the lines of its target-genome shard (crc32 of PAF column 6)
    batch = pw.HostBatch(fa, paf, flags, rank, world) if sharded else pw.HostBatch(fa, paf, flags)
    v = batch.view
    dev = pw.stage_batch(batch, dev_name)
    torch.cuda.synchronize()
    log(f"[rank {rank}] staged {v.n_alns} records, {v.n_ops} ops, {v.n_lits} literal bytes "
        f"({t_gen:.1f}s generate, {time.time() - t0 - t_gen:.1f}s pack + stage)")

    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    gtab = None
    if world > 1:
        # per-genome coverage / event tables (pw_genome_table) all-gathered every step (RCCL):
        # padded to the largest rank's row count, measured once here
        from pwasm_amd import mgpu
        rows, _, gt = mgpu.genome_rows(batch, dev, sp)
        if dist.get_backend() == "gloo":
            nb = torch.tensor([rows.numel()], dtype=torch.int64)
            nbs = [torch.empty_like(nb) for _ in range(world)]
            dist.all_gather(nbs, nb)
        else:
            nb = torch.tensor([rows.numel()], dtype=torch.int64, device=dev_name)
            nbs = [torch.empty_like(nb) for _ in range(world)]
            dist.all_gather(nbs, nb)
        pad = max(int(x.item()) for x in nbs)
        gtab = (mgpu, rows, gt, torch.zeros(max(pad, 16), dtype=torch.uint8, device=dev_name),
                torch.empty(world * max(pad, 16), dtype=torch.uint8, device=dev_name))

    # the next-stop table is built by the pass itself (PW_REPORT_BUILD_NEXT_STOP: index_kernel's
    # first workgroups, beside the decode) — round 5; before, a side stream built it and the pass
    # waited for its event before render.  PW_NS_SIDE=1 keeps that form (A/B sweeps).
    side_ns = os.environ.get("PW_NS_SIDE") == "1"
    side = torch.cuda.Stream()
    ns_ready, pass_done = torch.cuda.Event(), torch.cuda.Event()

    def step():
        ready = None
        a = pw.report_args(batch, dev)
        if not v.skip_codan and side_ns:
            side.wait_event(pass_done)
            rc = pw.lib().pw_stop_table_build(dev["qseq"].data_ptr(), dev["qoff"].data_ptr(), dev["qlen"].data_ptr(),
                                              int(v.n_queries), dev["next_stop"].data_ptr(), side.cuda_stream)
            assert rc == 0
            ns_ready.record(side)
            ready = ns_ready.cuda_event
        elif not v.skip_codan:
            a.flags |= pw.REPORT_BUILD_NEXT_STOP
        rc = pw.lib().pw_report_events_after(pw.ctypes.byref(a), sp, ready)
        assert rc == 0
        pass_done.record(stream)
        if gtab is not None:
            mg, rows, gt, padded, gathered = gtab
            mg.launch_genome_table(dev, rows, gt, sp)
            padded[: rows.numel()].copy_(rows)
            if dist.get_backend() == "gloo":  # (rehearsal only: host copies)
                h = [torch.empty(padded.numel(), dtype=torch.uint8) for _ in range(world)]
                dist.all_gather(h, padded.cpu())
            else:
                dist.all_gather_into_tensor(gathered, padded)

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()
    res = pw.results_array(dev["results"].cpu().numpy())[: v.n_alns]
    n_events = int(res["n_events"].sum())
    errs = int((res["err"] != 0).sum())
    text_bytes = int(res["text_len"].astype(np.int64).sum())
    if not os.environ.get("PW_BENCH_NOCHECK"):  # (set by attribution sweeps of variants that render wrong)
        assert errs == 0, f"{errs} records reported errors"
    ctr = dev["work"][:64].cpu().numpy().view(np.uint32)
    log(f"[rank {rank}] {n_events} events, {text_bytes} text bytes; long lines {int(ctr[1])}; "
        f"ctr[7:16] {ctr[7:16].tolist()}")  # (ctr[7:16]: zeros unless an experiment build counts there)

    # HIP events around the K passes as a whole (an event pair per pass would put two timestamp
    # packets, ~5 us of GPU time, between consecutive passes)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    t_el = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
    kern_ms = ev0.elapsed_time(ev1) / args.steps

    tot_events = n_events
    tot_records = int(v.n_alns)
    max_el = t_el
    red_dev = dev_name if dist.is_initialized() and dist.get_backend() != "gloo" else "cpu"
    if world > 1:
        t = torch.tensor([t_el], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        max_el = float(t.item())
        e = torch.tensor([n_events, int(v.n_alns)], dtype=torch.float64, device=red_dev)
        dist.all_reduce(e, op=dist.ReduceOp.SUM)
        tot_events = int(e[0].item())
        tot_records = int(e[1].item())
    e2e_node = None
    flags_cli = ["-G", "-C"] if flags else []
    pre_hash = None
    if sharded and world == 1 and not args.no_parity and not args.no_e2e:
        # (the benchmarked batch's report is hashed before the end-to-end leg releases its device
        # buffers; the rank-0 block below reuses the result)
        pre_hash = hash_parity(pw, batch, dev, flags_cli, fa, paf, tmp)
    if sharded and not args.no_e2e:
        # end to end over the node: pwasm_amd.mgpu (every rank reads 1/N of the PAF, exchanges lines
        # by target genome, packs / runs / writes its own records at their offsets of one report);
        # at N = 1 the same driver with one rank, so the N-rank walls divide by it
        from pwasm_amd import mgpu
        dev = None
        torch.cuda.empty_cache()
        out_path = os.path.join(shared, "report_e2e.txt")
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        code = mgpu.main(["-G", "-C", "-r", fa, paf, "-o", out_path])
        wall = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            wall = float(t.item())
        if rank == 0:
            e2e_node = {"wall_s": round(wall, 3), "events_per_s": tot_events / wall, "rc": code,
                        "cmd": f"torchrun x{world} -m pwasm_amd.mgpu -G -C -r q.fa a.paf -o report.txt "
                               f"({os.path.getsize(paf)} B in, {os.path.getsize(out_path)} B out)"}
            if args.e2e_parity:
                want = oracle_crc(["-G", "-C"], fa, paf, host_threads())
                with open(out_path, "rb") as f:
                    got = crc_stream(f)
                e2e_node["parity"] = "ok" if code == 0 and got == want[:3] else "FAIL"
            log(f"[e2e] {world} ranks: {wall:.2f} s, rc {code}")
        if world > 1:
            dist.barrier()

    if rank == 0:
        report = {}
        # algorithmic bytes of one pass, SURVEY.md §8(d): 16 B per record descriptor, 4 B per packed
        # op, 1 B per literal, 32 B per event record, 13 B per base of each distinct query (the base
        # + 3 frame next-stop int32 entries; 1 B when the codon pass is skipped, -F / -N)
        desc = batch.array("desc").view(np.uint32).reshape(-1, 8)
        qlen = batch.array("qlen").astype(np.int64)
        uq = np.unique(desc[:, 3] & 0x3FFFFFFF)
        per_base = 1 if v.skip_codan else 13
        alg_bytes = int(16 * v.n_alns + 4 * v.n_ops + v.n_lits + 32 * n_events + per_base * int(qlen[uq].sum()))
        # the report-text variant: inputs + the text actually written
        alg_text = int(v.alg_bytes_in) + text_bytes
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        prof = {}
        if config == 2 and args.scale == 1.0 and args.traffic_json and os.path.exists(args.traffic_json):
            prof = json.load(open(args.traffic_json))
        traffic = prof.get("hbm_bytes_per_report_pass", prof.get("hbm_bytes_per_launch"))
        parity, cpu, e2e, gpack = None, None, None, None
        big = config == 4 or v.n_alns > 200000
        if not args.no_parity and world == 1 and big:
            # too large for files on both sides: the report of the benchmarked batch and the
            # CLI's stdout streamed through CRC-32, against the oracle run over byte ranges of
            # the PAF in parallel processes with the CRCs combined (hash_parity)
            parity, e2e, n_or = pre_hash if pre_hash is not None else hash_parity(pw, batch, dev, flags_cli, fa,
                                                                                   paf, tmp)
            if n_or != n_events:
                parity = "FAIL"
        elif not args.no_parity and world == 1:
            # the benchmarked batch itself, copied back once (outside the timed region) and
            # diffed byte for byte against the oracle on the same input
            got = os.path.join(tmp, "hip.txt")
            rc = batch.write_report_from(dev, got)
            want = os.path.join(tmp, "oracle.txt")
            el = run_oracle(flags_cli, fa, paf, want)
            parity = "ok" if rc == 0 and filecmp.cmp(got, want, shallow=False) else "FAIL"
            n_or = count_events(want)
            if not args.no_cpu_baseline and (args.cpu_sample or v.n_alns) >= v.n_alns:
                cpu = {"value": n_or / el, "unit": "events/s", "cores": 1, "kind": "port",
                       "sample": f"the whole benchmarked batch ({v.n_alns} records, {n_or} events, {el:.1f} s, "
                                 f"oracle/pafreport_oracle pinned to one core)"}
            # end to end: the drop-in CLI (PAF text in, report file out) on the same input, three
            # runs after a sync (the oracle and parity legs before it leave ~0.6 GB of dirty page
            # cache, whose writeback throttled the CLI's writes: 0.19 vs 0.49 s on one box), the
            # median reported, every run listed
            cli_out = os.path.join(tmp, "cli.txt")
            runs, cli_ok = [], True
            for _ in range(3):
                os.sync()
                t0 = time.perf_counter()
                p = subprocess.run([str(REPO / "pwasm_amd/bin/pafreport"), *flags_cli, "-r", fa, paf, "-o", cli_out],
                                   stderr=subprocess.PIPE)
                runs.append(time.perf_counter() - t0)
                cli_ok = cli_ok and p.returncode == 0 and filecmp.cmp(cli_out, want, shallow=False)
            cli_s = sorted(runs)[1]
            e2e = {"cli_wall_s": round(cli_s, 3), "cli_wall_runs_s": [round(x, 3) for x in runs],
                   "events_per_s": n_or / cli_s, "parity": "ok" if cli_ok else "FAIL",
                   "cmd": f"pafreport {' '.join(flags_cli)} -r q.fa a.paf -o report.txt (PAF text -> report file, "
                          f"{os.path.getsize(paf)} B in, {os.path.getsize(want)} B out)",
                   "phases": cli_phases(flags_cli, fa, paf, os.path.join(tmp, "cli2.txt"))}
            if not cli_ok:
                parity = "FAIL"
            gpack = gpu_pack_check(pw, paf)
        if cpu is None and not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(flags_cli, fa, paf, args.cpu_sample if args.cpu_sample else
                               (10 if config == 4 else 100000), tmp)
        if cpu is not None:
            cpu.update(host_cpu())
        out = {
            "metric": "cs-events classified/sec (whole node) + achieved HBM GB/s, 1/2/4/8 MI355X",
            "value": tot_events * args.steps / max_el,
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": max_el * 1000.0 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (pwsynth, seeded minimap2-style PAF with cs/cg tags)",
            "config": {"workload": (f"cfg3: {tot_records} PAF records (gene panel of {v.n_queries} CDS x assemblies, "
                                    f"-G -C) sharded by target genome over {world} GPU(s), {tot_events} events"
                                    if sharded else
                                    f"cfg{config}: {v.n_alns} PAF records/GPU over {v.n_queries} CDS "
                                    f"({'-G -C' if flags else 'auto'}), {n_events} events/GPU"),
                       "records_per_gpu": int(v.n_alns), "events_per_gpu": n_events, "scale": args.scale,
                       "records_total": tot_records, "events_total": tot_events,
                       "parallelism": (f"shard-by-target x{world} + RCCL all-gather of per-genome tables"
                                       if sharded and world > 1 else
                                       ("independent per-rank batches (weak scaling: the same cfg2 work per "
                                        "GPU at every N; the strong-scaling figure is scaling_cfg3)"
                                        if world > 1 else "single GPU"))},
            "parity": parity,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel": "pw_report_events (index+tctx+render+fixup+finalize)", "kernel_ms": round(kern_ms, 4),
                         "alg_bytes_per_launch": alg_bytes,
                         "alg_formula": "SURVEY 8(d): 16*n_alns + 4*n_ops + n_lits + 32*E + 13*sum(L unique queries)",
                         "achieved_text_variant": round(alg_text / (kern_ms * 1e-3) / 1e9, 2),
                         "alg_bytes_text_variant": alg_text,
                         "occupancy_waves_per_simd": prof.get("occupancy_waves_per_simd"),
                         "issue_busy": issue_busy(prof, ("pw::render_kernel", "pw::index_kernel", "pw::tctx_kernel"))},
            "cpu_baseline": cpu,
            "e2e": e2e if e2e is not None else e2e_node,
            "gpu_pack": gpack,
        }
    dev = None
    if world > 1:
        dist.barrier()
    shutil.rmtree(tmp, ignore_errors=True)  # (rank 0's is the shared one at cfg3: ~4 GB of PAF + report)
    return out if rank == 0 else None


def bench_gapassem(args, world, rank, dev_name):
    """BASELINE.json configs[4]: GapAssem consensus of one 200-row, ~1M-column layout (pwsynth
    cfg5, seed 5), rows sharded over the ranks (strong scaling).  A step on one GPU =
    pw_msa_columns_refine (count, bestChar and, without removeConsGaps, the consensus string in
    one counting pass; with --remove-gaps + the pw_msa_refine kernels); on N > 1 = pw_msa_count on the
    rank's rows + pw_msa_call_sharded (RCCL reduce-scatter of the [n_cols x 6] histograms by
    column range + bounds, bestChar of the rank's columns, all-gather of the consensus) +
    pw_msa_refine (consensus string; with --remove-gaps also the removeConsGaps row edits).  Default removeConsGaps=false: pafreport's setting (pafreport.cpp:31,203), which is
    also what the linear-time CPU oracle can time at full size.  Throughput = layout bases per
    second (all rows, whole job)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from pwasm_amd import gapassem

    remove = bool(args.remove_gaps)
    tmp = tempfile.mkdtemp(prefix=f"pwga{rank}_")
    lay_path = os.path.join(tmp, "l.pwl")
    t0 = time.time()
    subprocess.run([str(REPO / "synth/build/pwsynth"), "layout", "--config", "5", "--scale", str(args.scale),
                    "--seed", "5", "--out", lay_path], check=True, stderr=subprocess.DEVNULL)
    hdr = gapassem.Layout(lay_path, load=set())
    lo, hi = gapassem.shard_rows(hdr.seqlen, world)[rank]
    lay = gapassem.Layout(lay_path, load=set(range(lo, hi)))
    eng = gapassem.HipEngine(dev_name)
    rccl = world > 1 and dist.get_backend() == "nccl"
    st = eng.stage(lay, range(lo, hi), lay.length, world if rccl else 1)
    comm = gapassem.rccl_comm() if rccl else None
    total_bases = int(hdr.seqlen.sum())
    log(f"[rank {rank}] layout {hdr.n} rows, {lay.length} columns, {total_bases} bases; rows [{lo},{hi}) "
        f"({time.time() - t0:.1f}s host prep)")
    mm = st["d"]["mm"]
    red = torch.empty(2, dtype=torch.int32, device=dev_name)

    def step():
        if world == 1:  # one shard: count + call (+ the consensus string) in one pass, then refine
            eng.columns_refine(st, remove)
            return
        counts, _ = eng.count(st)
        if rccl:  # column-sharded: reduce-scatter by column range, own-range bestChar, all-gather
            eng.call_sharded(st, lo, comm, rank, world)
            eng.refine(st, remove)
            return
        if world > 1:  # (gloo rehearsal: host all-reduce of the whole histogram)
            dist.all_reduce(counts, op=dist.ReduceOp.SUM)
            red[0] = mm[0]
            red[1] = -mm[1]
            dist.all_reduce(red, op=dist.ReduceOp.MIN)
            mm[0] = red[0]
            mm[1] = -red[1]
        eng.call(st)
        eng.refine(st, remove)

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()
    zero = int(mm[3].item())
    if not os.environ.get("PW_BENCH_NOCHECK"):  # (set by attribution sweeps of variants that count wrong)
        assert zero == 2 ** 31 - 1 and int(mm[2].item()) == 2 ** 31 - 1, "layout errors"
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)  # (around all K steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    t_el = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    max_el = t_el
    if world > 1:
        t = torch.tensor([t_el], dtype=torch.float64, device=dev_name)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        max_el = float(t.item())
    parity = None
    if not args.no_parity:
        # the whole layout through the same driver (outside the timed region): PWC1 bytes vs the
        # GapAssem oracle (refineMSA restated, GapAssem.cpp:1133-1198)
        rc, _, got = gapassem.consensus(lay_path, remove_gaps=remove)
    if rank == 0:
        cpu = None
        if not args.no_parity:
            want = os.path.join(tmp, "oracle.pwc")
            pin, cpu0 = pin_cmd()
            t0 = time.perf_counter()
            p = subprocess.run(pin + [str(REPO / "oracle/build/gapassem_oracle"), lay_path, want,
                                      *(["--remove-gaps"] if remove else [])])
            el = time.perf_counter() - t0
            parity = "ok" if rc == 0 and p.returncode == 0 and open(want, "rb").read() == got else "FAIL"
            if not args.no_cpu_baseline and not remove:
                cpu = {"value": total_bases / el, "unit": "bases/s", "cores": 1, "kind": "port",
                       "sample": f"the whole layout ({hdr.n} rows, {total_bases} bases, {el:.1f} s; "
                                 f"oracle/gapassem_oracle, removeConsGaps=false, pinned to cpu {cpu0})"}
        ncols = lay.length
        # algorithmic bytes: 16 B row descriptor + 3 B per base (base + int16
        # gap) read, 24 B counts + 1 B consensus per column written; this rank's rows
        own = int(lay.seqlen[lo:hi].sum())
        alg = 16 * (hi - lo) + 3 * own + 25 * ncols
        achieved = alg / (kern_ms * 1e-3) / 1e9
        prof = {}
        if args.traffic_json and os.path.exists(args.traffic_json) and args.scale == 1.0 and not remove:
            prof = json.load(open(args.traffic_json))
        out = {
            "metric": "GapAssem layout bases called/sec (count + histogram all-reduce + bestChar + refineMSA)",
            "value": total_bases * args.steps / max_el,
            "unit": "bases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": max_el * 1000.0 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (pwsynth layout cfg5, seed 5)",
            "config": {"workload": f"cfg5: {hdr.n} rows x {ncols} columns, {total_bases} bases, "
                                   f"removeConsGaps={'true' if remove else 'false'}",
                       "rows": int(hdr.n), "columns": int(ncols), "parallelism": f"rows sharded x{world}"},
            "parity": parity,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": prof.get("hbm_bytes_per_launch"),
                         "kernel": ("pw_msa_columns_refine" if world == 1 else "pw_msa_count+pw_msa_call+pw_msa_refine") + " (rank 0)", "kernel_ms": round(kern_ms, 4),
                         "alg_bytes_per_launch": alg,
                         "alg_formula": "SURVEY 8(d): sum_rows(16 + 3*seqlen) + 25*n_cols",
                         "occupancy_waves_per_simd": prof.get("occupancy_waves_per_simd"),
                         "issue_busy": issue_busy(prof, ("pw::tile_counts", "pw::row_chunk_sums"))},
            "cpu_baseline": cpu,
        }
        return out
    return None


def launch_plan(gpus, argv, env, port=None):
    """What `bench.py --gpus N` starts: [] when this process is the (only) rank itself; a list of
    (argv, env) pairs, one per rank, when it must launch N > 1 ranks (no WORLD_SIZE in the
    environment); an error string when WORLD_SIZE contradicts --gpus.  Pure: nothing is started and
    no GPU is touched (tests/test_bench_launch.py)."""
    world = env.get("WORLD_SIZE")
    if world is not None:
        if gpus is not None and int(world) != gpus:
            return f"WORLD_SIZE={world} but --gpus {gpus}: run one rank per GPU (torchrun --nproc-per-node {gpus})"
        return []
    if gpus is None or gpus <= 1:
        return []
    if port is None:
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
    plan = []
    for r in range(gpus):
        e = dict(env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(gpus), "LOCAL_WORLD_SIZE": str(gpus),
                  "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                  "PW_BENCH_LAUNCHER": "bench.py --gpus"})
        plan.append(([sys.executable, str(REPO / "bench.py"), *argv], e))
    return plan


def run_ranks(plan, poll_s=0.5):
    """Start every rank of the plan as a child process (same process group, inherited stdout /
    stderr: rank 0 prints the JSON line) and wait; the first rank that fails ends the others.
    Returns the exit code: 0, or the first failing rank's."""
    procs = [subprocess.Popen(cmd, env=env) for cmd, env in plan]
    code = 0
    try:
        while procs:
            for p in list(procs):
                rc = p.poll()
                if rc is None:
                    continue
                procs.remove(p)
                if rc != 0 and code == 0:
                    code = rc if rc > 0 else 128 - rc
                    log(f"bench.py: a rank exited with {rc}; stopping the others")
                    for q in procs:
                        q.terminate()
            time.sleep(poll_s)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
                q.wait()
    return code


def host_cpu():
    """CPU model and core counts of the host the baseline ran on."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}


def crc32_combine(crc1, crc2, len2):
    """zlib's crc32_combine (GF(2) matrix powers): the CRC-32 of A+B from crc(A), crc(B), len(B)."""
    def times(mat, vec):
        s, i = 0, 0
        while vec:
            if vec & 1:
                s ^= mat[i]
            vec >>= 1
            i += 1
        return s

    def square(mat):
        return [times(mat, mat[n]) for n in range(32)]

    if len2 <= 0:
        return crc1
    odd = [0xEDB88320] + [1 << n for n in range(31)]
    even = square(odd)
    odd = square(even)
    while True:
        even = square(odd)
        if len2 & 1:
            crc1 = times(even, crc1)
        len2 >>= 1
        if not len2:
            break
        odd = square(even)
        if len2 & 1:
            crc1 = times(odd, crc1)
        len2 >>= 1
        if not len2:
            break
    return crc1 ^ crc2


def crc_stream(f, block=1 << 22):
    """(crc32, bytes, event lines) of a binary stream read to its end."""
    import zlib
    crc, n, lines, hdr, tail = 0, 0, 0, 0, b"\n"
    while True:
        b = f.read(block)
        if not b:
            break
        crc = zlib.crc32(b, crc)
        n += len(b)
        lines += b.count(b"\n")
        hdr += b.count(b"\n>") + (tail == b"\n" and b[:1] == b">")
        tail = b[-1:]
    return crc, n, lines - hdr


def oracle_crc(flags_cli, fa, paf, procs, chunks_per_proc=4):
    """The oracle over the PAF in byte ranges (--range; --elide-dead skips the query-suffix copy
    nothing reads when the codon pass is off), `procs` processes at a time, each stdout streamed
    through CRC-32 and the CRCs combined in order.  A range split can only differ from one pass
    through the gene-mode q~t dedupe across ranges, which would show as a mismatch, never hide
    one.  Returns (crc, bytes, events, seconds)."""
    from concurrent.futures import ThreadPoolExecutor
    size = os.path.getsize(paf)
    k = max(1, procs * chunks_per_proc)
    cuts = [size * i // k for i in range(k + 1)]

    def one(i):
        p = subprocess.Popen([str(REPO / "oracle/build/pafreport_oracle"), "--elide-dead", "--range",
                              f"{cuts[i]}:{cuts[i + 1]}", *flags_cli, "-r", fa, paf],
                             stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
        r = crc_stream(p.stdout)
        if p.wait() != 0:
            raise RuntimeError(f"oracle range {i} failed")
        return r

    t0 = time.perf_counter()
    with ThreadPoolExecutor(procs) as ex:
        parts = list(ex.map(one, range(k)))
    crc, n, ev = 0, 0, 0
    for c, m, e in parts:
        crc = crc32_combine(crc, c, m)
        n += m
        ev += e
    return crc, n, ev, time.perf_counter() - t0


def hash_parity(pw, batch, dev, flags_cli, fa, paf, tmp):
    """Parity of a large run (cfg3 at 10M records, cfg4): the benchmarked batch's report (written
    by pw_batch_write_report into a FIFO) and the drop-in CLI's stdout (end to end, PAF text in)
    vs the chunked oracle, by CRC-32 + length + event count.  -> (parity, e2e, oracle events)."""
    import threading
    want = oracle_crc(flags_cli, fa, paf, host_threads())
    log(f"[parity] oracle: {want[1]} bytes, {want[2]} events in {want[3]:.1f}s ({host_threads()} processes)")
    fifo = os.path.join(tmp, "report.fifo")
    os.mkfifo(fifo)
    got = {}

    def reader():
        with open(fifo, "rb") as f:
            got["r"] = crc_stream(f)

    th = threading.Thread(target=reader, daemon=True)
    th.start()
    rc = -1
    try:
        rc = batch.write_report_from(dev, fifo)
    finally:
        if rc != 0 and "r" not in got:  # never opened (or failed first): release the reader
            open(fifo, "wb").close()
        th.join()
    batch_ok = rc == 0 and got.get("r") == want[:3]
    # the drop-in CLI writing its report to a local file (-o), timed alone; CRC-checked afterwards
    cli_out = os.path.join(tmp, "cli.txt")
    t0 = time.perf_counter()
    cli_rc = subprocess.run([str(REPO / "pwasm_amd/bin/pafreport"), *flags_cli, "-r", fa, paf, "-o", cli_out],
                            stderr=subprocess.DEVNULL).returncode
    cli_s = time.perf_counter() - t0
    with open(cli_out, "rb") as f:
        cli = crc_stream(f)
    os.remove(cli_out)
    cli_ok = cli_rc == 0 and cli == want[:3]
    e2e = {"cli_wall_s": round(cli_s, 3), "events_per_s": want[2] / cli_s, "parity": "ok" if cli_ok else "FAIL",
           "cmd": f"pafreport {' '.join(flags_cli)} -r q.fa a.paf -o report.txt (PAF text -> report file, "
                  f"{os.path.getsize(paf)} B in, {cli[1]} B out, CRC-32 checked after the run)"}
    log(f"[parity] batch report {'ok' if batch_ok else 'FAIL'} (crc {got.get('r')} vs {want[:3]}); "
        f"CLI {'ok' if cli_ok else 'FAIL'} {cli_s:.1f}s")
    parity = {"result": "ok" if batch_ok and cli_ok else "FAIL", "method": "CRC-32 + bytes + events, streamed",
              "oracle": f"oracle/pafreport_oracle over {host_threads() * 4} byte ranges, {host_threads()} processes, "
                        f"{want[3]:.1f}s", "bytes": want[1], "crc32": f"{want[0]:08x}"}
    return parity, e2e, want[2]


def cli_phases(flags_cli, fa, paf, outp):
    """A second CLI run with PW_PROFILE_HOST=1: its own phase timestamps (FASTA load, first batch read
    + pack, device init, per batch GPU run + result copies and emit, total), parsed from stderr, plus
    the two ends its own clock cannot see: `process_start` (spawn -> main's first instruction: exec,
    the dynamic loader and the HIP runtime library's static initialisers) and `exit` (the last
    instruction -> the parent has reaped it: the kernel's teardown of the process and its GPU
    state), from wall-clock epochs the CLI prints; `wall_s` is this run's own wall clock."""
    import re
    env = {**os.environ, "PW_PROFILE_HOST": "1"}
    os.sync()
    t_spawn = time.time()
    p = subprocess.run([str(REPO / "pwasm_amd/bin/pafreport"), *flags_cli, "-r", fa, paf, "-o", outp],
                       stderr=subprocess.PIPE, env=env)
    t_reaped = time.time()
    ph = {}
    for ln in p.stderr.decode(errors="replace").splitlines():
        if ln.startswith("[cli-dev]"):  # (the device side's steps, overlapped with the phases: not summed)
            ph["device_steps_at"] = {re.sub(r"[^a-z0-9]+", "_", k.strip()).strip("_"): float(v)
                                     for k, v in re.findall(r"([a-z][a-z +()\-]*?) at ([0-9.]+) s", ln[9:])}
            continue
        if not ln.startswith("[cli]"):
            continue
        m = re.match(r"\[cli\] (main_entry|exit)_epoch ([0-9.]+)", ln)
        if m:
            ph["process_start" if m.group(1) == "main_entry" else "exit"] = round(
                float(m.group(2)) - t_spawn if m.group(1) == "main_entry" else t_reaped - float(m.group(2)), 4)
            continue
        for name, val in re.findall(r"([a-z][a-z +()\-]*?) ([0-9.]+) s", ln[5:]):
            key = re.sub(r"[^a-z0-9]+", "_", name.strip()).strip("_")
            ph[key] = round(ph.get(key, 0.0) + float(val), 4)
    if ph:
        ph["wall_s"] = round(t_reaped - t_spawn, 4)
        ph["accounted_s"] = round(sum(ph.get(k, 0.0) for k in ("process_start", "total", "close_output", "teardown",
                                                                  "exit")), 4)
    try:
        os.remove(outp)
    except OSError:
        pass
    return ph or None


def rank_thread_share():
    """Under torchrun (which sets OMP_NUM_THREADS=1 when the caller left it unset) a rank's host
    pre-pass would run on one thread: with several ranks and no PW_THREADS, give each rank its share
    of this process's CPUs (at most 16) through PW_THREADS, which the library reads first."""
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")) or 1)
    if lw > 1 and not os.environ.get("PW_THREADS") and os.environ.get("OMP_NUM_THREADS") == "1":
        os.environ["PW_THREADS"] = str(max(1, min(16, len(os.sched_getaffinity(0)) // lw)))


def host_threads():
    for k in ("PW_THREADS", "OMP_NUM_THREADS"):
        if os.environ.get(k, "").isdigit() and int(os.environ[k]) > 0:
            return int(os.environ[k])
    return max(1, min(len(os.sched_getaffinity(0)), 16))


def gpu_pack_check(pw, paf, reps=10):
    """every cs string of the benchmarked PAF packed on the GPU (pw_pack_cs_batch,
    inputs resident, HIP events over `reps` launches) and compared record by record with the host
    packer pw_pack_cs (op words, literal bytes, totals)."""
    import numpy as np
    import torch
    cs, offs, qls = [], [], []
    for line in open(paf, "rb"):
        f = line.rstrip(b"\r\n").split(b"\t")
        if len(f) < 12 or line.startswith(b"#"):
            continue
        c = next((x[5:] for x in f[12:] if x.startswith(b"cs:Z:")), None)
        if c is None:
            continue
        ql, qs, qe = int(f[1]), int(f[2]), int(f[3])
        cs.append(c)
        offs.append(qs if f[4] == b"+" else ql - qe)
        qls.append(ql)
    ops, lits, off, recs = pw.pack_cs_gpu(cs, offs, qls)
    bad = 0
    for i in range(len(cs)):
        rc, hops, hlits, tot, _ = pw.pack_cs(cs[i].decode("latin-1"), offs[i], qls[i])
        g, b = recs[i], int(off[i])
        if g["flags"] & pw.PACK_HOST:
            bad += rc == 0
            continue
        same = (rc == 0 and list(ops[b: b + g["n_ops"]]) == hops and bytes(lits[b: b + g["n_lits"]]) == hlits
                and int(g["n_events_max"]) == tot.n_events_max and int(g["t_total"]) == tot.t_total)
        bad += not same
    # timing on device-resident inputs
    n = len(cs)
    o = np.zeros(n + 1, dtype=np.uint64)
    o[1:] = np.cumsum([len(c) for c in cs], dtype=np.uint64)
    t = lambda a: torch.from_numpy(np.array(a, copy=True)).cuda()
    d_text = t(np.frombuffer(b"".join(cs) + b"\0" * 16, dtype=np.uint8))
    d_off, d_o, d_q = t(o.view(np.int64)), t(np.asarray(offs, dtype=np.int32)), t(np.asarray(qls, dtype=np.int32))
    d_ops = torch.empty(int(o[-1]) + 16, dtype=torch.int32, device="cuda")
    d_lits = torch.empty(int(o[-1]) + 16, dtype=torch.uint8, device="cuda")
    d_rec = torch.empty(n * pw.CS_REC.itemsize, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    call = lambda: pw.lib().pw_pack_cs_batch(d_text.data_ptr(), d_off.data_ptr(), d_o.data_ptr(), d_q.data_ptr(), n,
                                             d_ops.data_ptr(), d_lits.data_ptr(), d_rec.data_ptr(), st.cuda_stream)
    call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        call()
    e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000.0 / reps
    return {"records": n, "cs_bytes": int(o[-1]), "us_per_batch": round(us, 1),
            "cs_GB_per_s": round(int(o[-1]) / us / 1e3, 1), "host_fallbacks": int((recs["flags"] & pw.PACK_HOST != 0).sum()),
            "parity": "ok" if bad == 0 else f"FAIL ({bad} records)"}


def issue_busy(prof, kernels, n_cu=256, n_xcd=8, simd_per_cu=4):
    """What bounds the report kernels instead of HBM, from the profile's PMC counters: the share of
    the kernel's cycles the SIMDs spend issuing VALU (a wave64 VALU instruction occupies a 32-lane
    CDNA4 SIMD for 2 cycles, MI355X_MICROARCH.md), the LDS is busy (SQ_LDS_IDX_ACTIVE, bank-conflict
    cycles included) and the per-CU texture address / data units are busy (TA_TA_BUSY, TD_TD_BUSY:
    the vector-memory pipeline, which scattered accesses load with one cache-line lookup per lane).
    GRBM_GUI_ACTIVE is summed over the XCDs."""
    pmc = prof.get("pmc_per_launch") or {}
    out = {}
    for k in kernels:
        c = pmc.get(k)
        if not c or not c.get("GRBM_GUI_ACTIVE"):
            continue
        cyc = c["GRBM_GUI_ACTIVE"] / n_xcd
        out[k] = {"valu_busy": round(2 * c.get("SQ_INSTS_VALU", 0) / (n_cu * simd_per_cu * cyc), 3),
                  "lds_busy": round(c.get("SQ_LDS_IDX_ACTIVE", 0) / (n_cu * cyc), 3)}
        for name, ctr in (("ta_busy", "TA_TA_BUSY_sum"), ("td_busy", "TD_TD_BUSY_sum")):
            if c.get(ctr):
                out[k][name] = round(c[ctr] / (n_cu * cyc), 3)
    return out or None


def latest_profile(config):
    """profiles/r<round>_v<k>/summary.json of the newest profile taken with this --config."""
    import re
    best, key = None, None
    for d in (REPO / "profiles").glob("r*_v*"):
        m = re.fullmatch(r"r(\d+)_v(\d+)", d.name)
        f = d / "summary.json"
        if not m or not f.exists():
            continue
        try:
            cfg = int(json.load(open(f)).get("config", 2))
        except (ValueError, OSError):
            continue
        k = (int(m.group(1)), int(m.group(2)))
        if cfg == config and (key is None or k > key):
            best, key = str(f), k
    return best


def pin_cmd():
    cpu0 = sorted(os.sched_getaffinity(0))[0]
    return (["taskset", "-c", str(cpu0)] if shutil.which("taskset") else []), cpu0


def run_oracle(flags_cli, fa, paf, outp):
    """The single-threaded oracle (C restatement of pafreport) on one core; returns seconds."""
    pin, _ = pin_cmd()
    t0 = time.perf_counter()
    subprocess.run(pin + [str(REPO / "oracle/build/pafreport_oracle"), *flags_cli, "-r", fa, paf, "-o", outp],
                   check=True)
    return time.perf_counter() - t0


def count_events(path):
    lines = hdr = 0
    with open(path, "rb") as f:
        for line in f:
            lines += 1
            hdr += line.startswith(b">")
    return lines - hdr


def cpu_baseline(flags_cli, fa, paf, n_rec, tmp):
    """Time the single-threaded oracle on the first n_rec records."""
    sample = os.path.join(tmp, "sample.paf")
    with open(paf) as f, open(sample, "w") as g:
        for i, line in enumerate(f):
            if i >= n_rec:
                break
            g.write(line)
    outp = os.path.join(tmp, "cpu.txt")
    el = run_oracle(flags_cli, fa, sample, outp)
    ev = count_events(outp)
    _, cpu0 = pin_cmd()
    return {"value": ev / el, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": f"first {n_rec} records of the same batch ({ev} events, {el:.1f} s, pinned to cpu {cpu0})"}


if __name__ == "__main__":
    main()
