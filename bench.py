#!/usr/bin/env python3
"""Benchmark of the CGNN neural-receiver forward pass on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Without a launcher, ``--gpus N > 1`` starts the N rank processes itself (a parent that never
touches the GPU spawns them with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, waits, and
exits with the worst rank's code), so ``python bench.py --gpus 8`` measures 8 ranks; under a
launcher WORLD_SIZE must equal --gpus.

Workload (BASELINE.json configs[1]): nrx_rt weights, 2 users, 4 PRB (F = 48), 4 rx
antennas, 16-QAM, batch 128 slots per GPU, f16 perf mode.  A "step" = one full CGNN
forward (norm, StateInit, 2 x [aggregation, state update], readouts) over the batch,
inputs already resident in HBM.  Multi-GPU: each rank runs its own 128-slot shard
(independent slots, no collective on the data path -> weak scaling); one RCCL
all-reduce of the per-rank elapsed time (MAX) after the timed region.

Prints ONE JSON line (rank 0) with the headline metric (slots/s, whole job), the
per-slot p50 latency at batch 1, the roofline of the dominant kernel
(the one-launch forward k_forward at this shape -- the state-update launch where the
three-launch path runs -- measured with HIP events on the launch stream) and a CPU baseline
(the torch-CPU restatement, fp32, BASELINE.md's plan: cfg1 latency and cfg2 throughput at
all threads and at 1 thread, on a bounded sample on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default="nrx_rt")
    p.add_argument("--batch", type=int, default=128, help="slots per GPU per step")
    p.add_argument("--users", type=int, default=2)
    p.add_argument("--prbs", type=int, default=4)
    p.add_argument("--precision", default="f16", choices=["f16", "f32x"])
    p.add_argument("--latency-iters", type=int, default=1000)
    p.add_argument("--prewarm-s", type=float, default=0.3,
                   help="seconds of untimed forwards before the W warmup steps (GPU clock ramp)")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-latency", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the generate+receive+count measurement")
    p.add_argument("--graph", action="store_true",
                   help="time replays of a captured hipGraph instead of direct nrx_forward calls")
    p.add_argument("--streams", type=int, default=2,
                   help="consecutive batches alternate over this many HIP streams, one engine (handle + "
                        "workspace + outputs) each, so a kernel's last waves overlap the next batch's "
                        "launch (1: one stream; --graph and --profile-only use one)")
    p.add_argument("--profile-only", action="store_true",
                   help="run warmup + timed steps only (for rocprofv3)")
    p.add_argument("--selftest", action="store_true",
                   help="launcher / timing / reduction plumbing only, on the CPU over gloo (no GPU "
                        "work, no engine): the line it prints is marked and is not a measurement")
    return p.parse_args()


def spawn_ranks(n: int) -> int:
    """--gpus N without a launcher: N child processes, one per GPU, started before this
    process touches the GPU (it never does); returns the worst exit code.  Only rank 0
    writes to stdout (the one JSON line)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = None if r == 0 else subprocess.DEVNULL
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env, stdout=out))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def selftest(args, world, rank):
    """Plumbing check of the multi-rank path on the CPU (gloo): barrier + timed region + MAX
    of the elapsed time + whole-job slot count, with a stand-in step (no GPU, no engine)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    x = torch.ones(64, 64)
    step = lambda: x @ x
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    slots_total = world * args.batch * args.steps
    if rank == 0:
        print(json.dumps({"metric": "selftest (launcher plumbing only, not a measurement)", "value":
                          round(slots_total / elapsed, 1), "unit": "slots/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "slots_total": slots_total, "data": "selftest",
                          "ranks_spawned_by": os.environ.get("NRX_BENCH_SPAWNED", "launcher")}))
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        os.environ["NRX_BENCH_SPAWNED"] = "bench.py"
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU is required")
    if args.selftest:
        selftest(args, world, rank)
        return
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    device = local_rank if world > 1 else 0
    torch.cuda.set_device(device)
    dev = f"cuda:{device}"

    from neural_rx_amd import metrics, synth
    from neural_rx_amd import weights as W
    from neural_rx_amd.config import dmrs_symbols, get_config, spec_from_config, user_cdm_groups
    from neural_rx_amd.receiver import CGNNEngine, compute_pe

    cfg = get_config(args.config)
    spec = spec_from_config(cfg)
    groups = user_cdm_groups(cfg, args.users)
    F = 12 * args.prbs
    B, U = args.batch, args.users
    num_it = cfg.num_nrx_iter_eval
    bits = [spec.bits[0]] * U
    slots = synth.generate(B, U, args.prbs, spec.num_rx_ant, bits, groups, dmrs_symbols(cfg),
                           snr_db=10.0, seed=1234 + 2 + 1000 * rank)
    pe_np = compute_pe(U, F, dmrs_symbols(cfg), groups)
    eng = CGNNEngine(spec, W.load(cfg.label), device)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)
    y, h, act, pe = t(slots.y), t(slots.h_hat), t(slots.active), t(pe_np)
    out = eng.alloc_outputs(B, U, F)
    # the throughput pipeline: batch i runs on stream i % S with engine i % S (each engine owns
    # its handle, workspace and outputs, so two batches in flight share no buffer); every batch
    # is a whole forward, only the launch boundaries of consecutive batches overlap
    n_streams = 1 if (args.graph or args.profile_only) else max(1, args.streams)
    engs = [eng] + [CGNNEngine(spec, W.load(cfg.label), device) for _ in range(n_streams - 1)]
    outs = [out] + [e.alloc_outputs(B, U, F) for e in engs[1:]]
    pipe_streams = [torch.cuda.Stream(device=dev) for _ in range(n_streams)]
    pipe_i = [0]

    def step_pipe():
        j = pipe_i[0] % n_streams
        pipe_i[0] += 1
        engs[j].forward(y, pe, h, act, None, num_it, args.precision, out=outs[j],
                        stream=pipe_streams[j].cuda_stream)
        fwd_count[0] += 1

    fwd_count = [0]   # forwards executed (--profile-only reports it: PMC records per forward)

    def step_eager():
        eng.forward(y, pe, h, act, None, num_it, args.precision, out=out)
        fwd_count[0] += 1

    # The timed steps are direct nrx_forward calls (async, no host sync: the host runs ahead
    # of the device); --graph replays one captured forward instead (measured slower at this
    # batch: a replay costs more than three back-to-back launches).
    graph_stream = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(graph_stream):
        for _ in range(max(args.warmup, 3)):
            step_eager()
    torch.cuda.synchronize()
    if not args.graph:
        step = step_pipe if n_streams > 1 else step_eager
    else:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=graph_stream):
            step_eager()
        torch.cuda.synchronize()
        fwd_count[0] -= 1   # captured, not executed

        def step():
            graph.replay()
            fwd_count[0] += 1

    # Steady state: the GPU takes tens of ms of back-to-back work to reach its load clock
    # (a fresh box measured 768 k slots/s with only the W = 5 warmup steps before 20 timed
    # ones, 920 k after 0.1 s of work, same binary); run untimed forwards for prewarm_s first.
    t_pw = time.perf_counter()
    while time.perf_counter() - t_pw < args.prewarm_s:
        for _ in range(50):
            step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    for e in engs:
        e.fused_status(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    fused_st = eng.fused_status(full=True)   # one-launch forward: prefetch misses in the timed region
    for e in engs[1:]:
        st_e = e.fused_status(full=True)
        fused_st = {"error": fused_st["error"] | st_e["error"], "waited": fused_st["waited"] + st_e["waited"],
                    "polls": fused_st["polls"] + st_e["polls"]}
    # one stream's own clock over a region of the same length (no per-launch markers): the step
    # time the per-launch event-pair shares below are scaled to, so the per-kernel durations are
    # those of kernels that do not overlap another batch's
    with torch.cuda.stream(graph_stream):
        ev_t0, ev_t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev_t0.record()
        for _ in range(args.steps):
            (step if n_streams == 1 else step_eager)()
        ev_t1.record()
    torch.cuda.synchronize()
    stream_step_ms = ev_t0.elapsed_time(ev_t1) / args.steps
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    if args.profile_only:
        if rank == 0:
            print(json.dumps({"profile_only": True, "ms_per_step": 1e3 * elapsed / args.steps,
                              "forwards": fwd_count[0]}))
        if world > 1:
            dist.destroy_process_group()
        return
    slots_total = world * B * args.steps
    value = slots_total / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # ---- roofline of the dominant kernel: HIP events around each launch, on the
    # launch stream, over a second timed region of the same length
    kflops = metrics.launch_flops_per_re_user(spec, num_it)
    re_users = B * U * F * 14
    eng.profile(True)
    for _ in range(args.steps):
        step_eager()
    prof = eng.profile_read()
    eng.profile(False)
    # An event pair around every launch adds a marker packet (~3 us) to each launch, so the
    # pairs are used for each kernel's SHARE of a step only; the shares are applied to the
    # step time of the uninstrumented region above (HIP events on the same stream).  This
    # agrees with the rocprofv3 kernel-trace average (profiles/r02/kernel_stats_v18.csv:
    # raw pairs 49.6 us vs trace 46.4 us; scaled 46.3 us).
    ev_step_ms = sum(ms for (n, ms) in prof.values() if n) / args.steps
    scale = min(1.0, stream_step_ms / ev_step_ms) if ev_step_ms > 0 else 1.0
    kern = {}
    for name, (n, ms) in prof.items():
        if n:
            avg_s = ms / n * 1e-3 * scale
            fl = kflops[name] * re_users
            kern[name] = {"launches": n, "avg_us": round(avg_s * 1e6, 3),
                          "avg_us_event_pairs": round(ms / n * 1e3, 3),
                          "tflops": round(fl / avg_s / 1e12, 2) if fl else None}
    fused_name = "forward_col" if prof.get("forward_col", (0, 0.0))[0] > 0 else "forward"
    fused = prof.get(fused_name, (0, 0.0))[0] > 0
    # the dominant kernel: the one-launch forward when the engine took it (throughput tier),
    # else the state-update launches of the three-launch forward, whichever kernel ran each
    # stage (nrx_update_schedule: the RR launch for the aggregation updates and the strip
    # k_update for the readout update by default) -- averaged over all update launches, as
    # kflops["state_update"] is the average work of one update launch
    if fused:
        dom, upd = fused_name, [fused_name]
    else:
        upd = [k for k in ("state_update_col", "state_update_rr", "state_update") if prof.get(k, (0, 0.0))[0]]
        dom = "state_update"
    dom_n = sum(prof[k][0] for k in upd)
    dom_ms = sum(prof[k][1] for k in upd)
    dom_avg_s = dom_ms / dom_n * 1e-3 * scale
    dom_flops = kflops[dom] * re_users
    peak = metrics.PEAK_TFLOPS[args.precision]
    achieved = dom_flops / dom_avg_s / 1e12
    elem = 2 if args.precision == "f16" else 4
    # algorithmic bytes = SURVEY 8(d)'s compulsory I/O of one forward (y, h_hat in; LLRs, h_ref
    # out; f32 as the ABI moves them); the schedule's own state hand-offs between stages are
    # reported separately (schedule_bytes_per_launch), never as algorithmic
    compulsory = metrics.compulsory_bytes_per_forward(spec, B, U, F, with_h=True)
    if fused:
        alg_bytes = metrics.forward_bytes_per_re_user(spec, num_it, U, elem) * re_users
        pmc_field, kname = "k_forward_bytes_per_launch", (
            "k_fwd_col (StateInit + num_it state updates + readouts as column items: one persistent launch)"
            if fused_name == "forward_col" else
            "k_forward (StateInit + num_it state updates + readouts: one persistent launch)")
        mixed = metrics.forward_mixed_bound_tflops(spec, num_it, peak) if args.precision == "f16" else None
        mixed_note = ("the forward's depthwise FLOPs at the VALU peak (157 TF) + its dense FLOPs at the "
                      "f16 MFMA peak, pipes overlapped (metrics.forward_mixed_bound_tflops)")
    else:
        alg_bytes = metrics.update_launch_bytes_per_re_user(spec, num_it, elem) * re_users
        names = {"state_update_col": "k_update_col (whole-column)", "state_update_rr": "k_update_rr (register-resident)",
                 "state_update": "k_update (strip)"}
        split = ", ".join(f"{names[k]} x {prof[k][0] // args.steps}" for k in upd)
        pmc_field, kname = "k_update_bytes_per_launch", (
            f"update stage (3 sep-convs + fused aggregation/readout tail; per forward: {split})")
        mixed = metrics.mixed_bound_tflops(spec, num_it, peak) if args.precision == "f16" else None
        mixed_note = ("k_update's depthwise FLOPs at the VALU peak (157 TF) + its dense FLOPs at the f16 "
                      "MFMA peak, pipes overlapped (metrics.mixed_bound_tflops)")
    traffic = None
    pmc, key = {}, f"{args.config}_b{B}_u{U}_p{args.prbs}_{args.precision}"
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            traffic = pmc.get(key, {}).get(pmc_field)
        except Exception:
            traffic = None
    pmc_src = None
    if traffic is not None:
        pmc_src = pmc.get(key, {}).get("source")
    # three launches: the whole forward's traffic (sum over its launches) beside the per-launch one
    fwd_traffic = None if fused else pmc.get(key, {}).get("forward_bytes")
    # SQ counters of the dominant kernel from the committed PMC capture (tools/pmc_record.py)
    sq = {}
    sq_path = os.path.join(ROOT, "profiles", "pmc_sq.json")
    if os.path.exists(sq_path):
        try:
            sq = json.load(open(sq_path)).get(key, {}).get(
                ("k_fwd_col" if fused_name == "forward_col" else "k_forward") if fused else "k_update", {})
        except Exception:
            sq = {}
    # counters are quoted only from a capture of the library that is running:
    # every record carries the nrx_build_id() of the library it profiled
    from neural_rx_amd import _lib
    build_id = _lib.load().nrx_build_id().decode()
    tr_rec = pmc.get(key, {})
    match = bool(sq) and sq.get("build_id") == build_id and (traffic is None and fwd_traffic is None
                                                             or tr_rec.get("build_id") == build_id)
    if not match:
        traffic = fwd_traffic = pmc_src = None
        sq = {k: v for k, v in sq.items() if k in ("source", "build_id")}
    whole_tflops = metrics.forward_flops_per_re_user(spec, num_it) * re_users * world / (elapsed / args.steps) / 1e12
    roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "kernel": kname,
                "flops_per_launch": dom_flops,
                "algorithmic_bytes_per_launch": compulsory if fused else None,
                "algorithmic_bytes_kind": "compulsory I/O of the forward (SURVEY 8(d): y, h_hat in, f32 LLRs "
                                          "and h_ref out, pe once)",
                "traffic_over_compulsory": round(traffic / compulsory, 3) if (traffic and fused) else (
                    round(fwd_traffic / compulsory, 3) if fwd_traffic else None),
                "compulsory_bytes_per_forward": compulsory,
                "traffic_per_forward": traffic if fused else fwd_traffic,
                "schedule_bytes_per_launch": round(alg_bytes),
                "schedule_bytes_kind": "the schedule's own hand-offs: StateInit reads y, h_hat and writes s, "
                                       "act*sp; every update reads s, a and writes s', act*sp or the outputs",
                "mfma_busy_frac": sq.get("mfma_busy_frac"),
                "valu_issue_frac": sq.get("valu_issue_frac"),
                "wait_frac": sq.get("wait_frac"),
                "sq_source": sq.get("source"),
                "avg_launch_us": round(dom_avg_s * 1e6, 3),
                "avg_launch_us_event_pairs": round(dom_ms / dom_n * 1e3, 3),
                "avg_launch_us_kind": "derived: event-pair share of a step x uninstrumented step time",
                "event_pair_scale": round(scale, 5),
                "uninstrumented_step_ms": round(stream_step_ms, 5),
                "timing": "per-launch HIP event pairs give each kernel's share of a step; "
                          "shares x the uninstrumented step time (HIP events, same stream); both regions "
                          "run on ONE stream, so these are the durations of kernels that overlap nothing "
                          "(value / ms_per_step come from the pipelined region)",
                "whole_forward_tflops": round(whole_tflops, 2),
                "whole_forward_frac": round(whole_tflops / world / peak, 4),
                "mixed_bound_tflops": round(mixed, 1) if mixed else None,
                "frac_of_mixed_bound": round(achieved / mixed, 4) if mixed else None,
                "mixed_bound_note": mixed_note,
                "traffic_source": pmc_src,
                "build_id": build_id,
                "counters_build_id": sq.get("build_id"),
                "counters_match_build": match}
    if fused:
        upd_items = args.steps * num_it * U * B * (((F + 23) // 24) if fused_name == "forward" else
                                                   (1 if F <= 48 else (F + 43) // 44))
        roofline["fused_queue"] = {"update_items_waited": fused_st["waited"], "update_items": upd_items,
                                   "polls": fused_st["polls"], "error": fused_st["error"],
                                   "ok": fused_st["waited"] == 0 and fused_st["error"] == 0,
                                   "note": "update items whose inputs were not complete when the previous item "
                                           "polled (z image loaded after a wait, not during that item's epilogue); "
                                           "ok = no wait and no error"}
        if fused_st["error"]:
            print(f"bench.py: one-launch forward error bits {fused_st['error']}: outputs invalid", file=sys.stderr)

    _progress(f"timed region done: {value:.0f} slots/s")
    # ---- batch-1 per-slot latency (hipGraph replay; device-only and H2D+compute+D2H)
    latency = None
    if not args.no_latency and rank == 0:
        latency = measure_latency(torch, eng, spec, cfg, args, groups, dev, num_it)
        latency["132prb_aerial_contract"] = measure_latency_aerial(torch, eng, spec, cfg, args, groups, dev, num_it)

    _progress("latency done")
    # ---- end-to-end Monte-Carlo step on the GPU: generate + receive + count (not `value`)
    e2e = None
    if not args.no_e2e:
        e2e = measure_e2e(torch, eng, spec, cfg, args, dev, num_it, rank, world)

    # ---- CPU baseline: the numpy oracle (fp32) on a bounded sample of the same workload
    cpu = None
    if not args.no_cpu_baseline and rank == 0 and world == 1:
        cpu = cpu_baseline(spec, cfg, slots, pe_np, args, num_it)

    if rank == 0:
        line = {
            "metric": "5G NR slots/sec + p50 per-slot latency, nrx_rt config",
            "value": round(value, 1),
            "unit": "slots/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f16" if args.precision == "f16" else "f32/f64",
            "data": "synthetic (seeded PUSCH slots: 16-QAM, DMRS type 1, TDL channel, LS+NN h_hat; trained nrx_rt weights)",
            "config": {"workload": f"{args.config}, {U} users, {args.prbs} PRB, 4 rx_ant, 16-QAM, "
                                   f"batch={B} slots per GPU",
                       "global_batch": B * world, "num_it": num_it, "parallelism": f"dp{world} (slot shards)",
                       "launch": "hipGraph replay of nrx_forward" if args.graph else (
                           "direct nrx_forward calls" if n_streams == 1 else
                           f"direct nrx_forward calls, consecutive batches alternated over {n_streams} HIP "
                           f"streams (one engine: handle + workspace + outputs each; every batch a whole forward)"),
                       "streams": n_streams,
                       "prewarm_s": args.prewarm_s},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "p50_latency_ms": latency,
            "e2e_generate_receive_count": e2e,
            "whole_forward_tflops": round(whole_tflops, 2),
            "kernels": kern,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def measure_e2e(torch, eng, spec, cfg, args, dev, num_it, rank, world):
    """One evaluation-loop step per batch, all on the GPU (neural_rx_amd.evaluate.sim_ber):
    the slot generator (nrx_generate_slots: bits, QAM, TDL channel, AWGN, LS+NN h_hat),
    the CGNN forward and the uncoded error counters (nrx_count_errors).  Same batch/shape as
    the headline; each rank generates its own slots (global slot index), no collective in
    the timed loop.  Reported beside the headline, never as `value`."""
    from neural_rx_amd.generator import GenParams, SlotGenerator, count_errors, ebno_to_no
    from neural_rx_amd.receiver import compute_pe
    B, U = args.batch, args.users
    p = GenParams.from_config(cfg, num_tx=U, num_prbs=args.prbs)
    gen = SlotGenerator(p, device=int(dev.split(":")[1]))
    no = ebno_to_no(4.0)
    pe = torch.from_numpy(compute_pe(U, p.num_subcarriers, p.dmrs_symbols, p.cdm_group)).to(dev)
    out = eng.alloc_outputs(B, U, p.num_subcarriers, want_h=False)
    counts = torch.zeros((U, 4), dtype=torch.int64, device=dev)

    def one(i):
        sb = gen(B, no, slot_offset=(i * world + rank) * B)
        llr, _ = eng.forward(sb.y, pe, sb.h_hat, sb.active, None, num_it, args.precision, out=out, want_h=False)
        count_errors(llr, sb.bits, sb.active, sb.mcs, p.mcs_bits, p.dmrs_symbols, counts=counts)

    for i in range(args.warmup):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        one(args.warmup + i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t1 = time.perf_counter()
    for i in range(args.steps):
        gen(B, no, slot_offset=i * B)
    torch.cuda.synchronize()
    gen_el = time.perf_counter() - t1
    c = counts.sum(0).cpu().numpy()
    return {"slots_per_s_per_gpu": round(B * args.steps / el, 1), "ms_per_step": round(1e3 * el / args.steps, 4),
            "generator_ms_per_batch": round(1e3 * gen_el / args.steps, 4), "ebno_db": 4.0,
            "uncoded_ber": float(c[0] / c[1]) if c[1] else None,
            "note": "GPU slot generator + CGNN forward + error counters per step (evaluate.sim_ber)"}


def measure_latency(torch, eng, spec, cfg, args, groups, dev, num_it):
    from neural_rx_amd import synth
    from neural_rx_amd.config import dmrs_symbols
    from neural_rx_amd.receiver import compute_pe
    res = {}
    for tag, prbs in (("4prb", args.prbs), ("132prb_trt_shape", 132)):
        F = 12 * prbs
        U = args.users
        s = synth.generate(1, U, prbs, spec.num_rx_ant, [spec.bits[0]] * U, groups,
                           dmrs_symbols(cfg), snr_db=10.0, seed=77)
        pe = torch.from_numpy(compute_pe(U, F, dmrs_symbols(cfg), groups)).to(dev)
        hy = torch.from_numpy(s.y).pin_memory()
        hh = torch.from_numpy(s.h_hat).pin_memory()
        ha = torch.from_numpy(s.active).pin_memory()
        y = hy.to(dev)
        h = hh.to(dev)
        a = ha.to(dev)
        out = eng.alloc_outputs(1, U, F)
        host_llr = torch.empty(out[0].shape, dtype=torch.float32).pin_memory()
        stream = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(stream):
            for _ in range(3):
                eng.forward(y, pe, h, a, None, num_it, args.precision, out=out)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            eng.forward(y, pe, h, a, None, num_it, args.precision, out=out)
        torch.cuda.synchronize()
        n = args.latency_iters
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        with torch.cuda.stream(stream):
            for i in range(n):
                ev[i][0].record(stream)
                g.replay()
                ev[i][1].record(stream)
        torch.cuda.synchronize()
        dev_ms = np.array([a_.elapsed_time(b_) for a_, b_ in ev])
        e2e = []
        with torch.cuda.stream(stream):
            for i in range(n):
                t0 = time.perf_counter()
                y.copy_(hy, non_blocking=True)
                h.copy_(hh, non_blocking=True)
                a.copy_(ha, non_blocking=True)
                g.replay()
                host_llr.copy_(out[0], non_blocking=True)
                stream.synchronize()
                e2e.append(time.perf_counter() - t0)
        e2e = np.array(e2e) * 1e3
        res[tag] = {"device_p50": round(float(np.median(dev_ms)), 4),
                    "e2e_p50": round(float(np.median(e2e)), 4),
                    "e2e_p99": round(float(np.percentile(e2e, 99)), 4),
                    "batch1_slots_per_s_e2e": round(1e3 / float(np.median(e2e)), 1)}
    return res


def measure_latency_aerial(torch, eng, spec, cfg, args, groups, dev, num_it, prbs=132):
    """Batch-1 latency of the Aerial / TensorRT contract (NeuralReceiverONNX I/O: raw rx
    grid + LS pilots in, Aerial-layout LLRs + refined h_hat out; FOCC, NN interpolation and
    PE on the GPU) at the reference TRT engine's shape (nrx_rt, 2 UE, 132 PRB).  e2e = H2D of
    every input + compute + D2H of both outputs, as trtexec's 1.409 ms median includes."""
    from neural_rx_amd import synth
    from neural_rx_amd.config import dmrs_symbols
    U = args.users
    syms = list(dmrs_symbols(cfg))
    s = synth.generate(1, U, prbs, spec.num_rx_ant, [spec.bits[0]] * U, groups, syms, snr_db=10.0, seed=78)
    yc = np.transpose(s.y_complex[:, 0], (0, 3, 2, 1))
    h_re, h_im = synth.aerial_ls_pilots(yc, s.x, groups, syms, prbs)
    host = {"y_real": np.ascontiguousarray(yc.real, np.float32), "y_imag": np.ascontiguousarray(yc.imag, np.float32),
            "h_ls_real": h_re, "h_ls_imag": h_im, "dmrs_port_mask": s.active}
    hp = {k: torch.from_numpy(np.ascontiguousarray(v)).pin_memory() for k, v in host.items()}
    d = {k: v.to(dev) for k, v in hp.items()}
    ofdm = torch.tensor([syms] * U, dtype=torch.int32, device=dev)
    scp = torch.tensor([[g + 2 * j for j in range(6)] for g in groups], dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(device=dev)
    call = lambda: eng.forward_aerial(d["y_real"], d["y_imag"], d["h_ls_real"], d["h_ls_imag"], d["dmrs_port_mask"],
                                      ofdm, scp, num_it, args.precision)
    with torch.cuda.stream(stream):
        for _ in range(3):
            call()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        llr, h = call()
    torch.cuda.synchronize()
    host_llr = torch.empty(llr.shape, dtype=torch.float32).pin_memory()
    host_h = torch.empty(h.shape, dtype=torch.float32).pin_memory()
    n = args.latency_iters
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    with torch.cuda.stream(stream):
        for i in range(n):
            ev[i][0].record(stream)
            g.replay()
            ev[i][1].record(stream)
    torch.cuda.synchronize()
    dev_ms = np.array([a_.elapsed_time(b_) for a_, b_ in ev])
    e2e = []
    with torch.cuda.stream(stream):
        for i in range(n):
            t0 = time.perf_counter()
            for k in d:
                d[k].copy_(hp[k], non_blocking=True)
            g.replay()
            host_llr.copy_(llr, non_blocking=True)
            host_h.copy_(h, non_blocking=True)
            stream.synchronize()
            e2e.append(time.perf_counter() - t0)
    e2e = np.array(e2e) * 1e3
    return {"shape": f"llr {tuple(llr.shape)}, h_hat {tuple(h.shape)}",
            "device_p50": round(float(np.median(dev_ms)), 4),
            "e2e_p50": round(float(np.median(e2e)), 4),
            "e2e_p99": round(float(np.percentile(e2e, 99)), 4),
            "batch1_slots_per_s_e2e": round(1e3 / float(np.median(e2e)), 1)}


def _progress(msg):
    """one stderr line per bench phase (a long silent phase looks hung to a supervisor)"""
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)


def cpu_quota():
    """CPUs this process may use: the affinity set, capped by a cgroup CPU quota when one is set
    (a box may expose every host CPU to the affinity mask while its cgroup grants a share of them;
    one torch thread per exposed CPU then oversubscribes the share many times over)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    return (min(n, quota) if quota else n), n, quota


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def cpu_baseline(spec, cfg, slots, pe_np, args, num_it):
    """BASELINE.md's CPU-baseline plan: the torch-CPU restatement of the CGNN
    (oracle/cgnn_torch.py: conv2d(groups=C) depthwise + 1x1 conv, fp32) on this host, at
    cfg 1 (1 UE, B = 1: p50 latency) and cfg 2 (the bench workload, B = 128: slots/s),
    with all the threads torch uses here and with 1 thread.  Identical seeded inputs to
    the GPU run.  The reference's own TF-CPU path cannot run (TensorFlow/Sionna absent)."""
    import torch
    from oracle import cgnn_ref
    from oracle.cgnn_torch import TorchCGNN
    from neural_rx_amd import synth
    from neural_rx_amd import weights as W
    from neural_rx_amd.config import dmrs_symbols, user_cdm_groups
    from neural_rx_amd.receiver import compute_pe
    model = TorchCGNN(cgnn_ref.split_keras_weights(W.load(cfg.label), spec), spec)
    # torch.set_num_threads(os.cpu_count()) -- here the CPUs this process may run on:
    # the affinity set, capped by the cgroup CPU quota (cpu_quota)
    torch_default = torch.get_num_threads()
    all_threads, affinity, quota = cpu_quota()
    B, U = slots.y.shape[0], slots.h_hat.shape[1]
    ones = lambda b, u: np.ones((b, u, spec.num_mcs), np.float32)
    # cfg 1: one user, batch 1 (same trained weights, 4 PRB)
    g1 = user_cdm_groups(cfg, 1)
    s1 = synth.generate(1, 1, args.prbs, spec.num_rx_ant, [spec.bits[0]], g1, dmrs_symbols(cfg), snr_db=10.0, seed=1235)
    pe1 = compute_pe(1, 12 * args.prbs, dmrs_symbols(cfg), g1)

    def p50_b1(n):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            model.forward(s1.y, pe1, s1.h_hat, s1.active, ones(1, 1), num_it)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts[2:])) * 1e3

    def b128(reps):
        t0 = time.perf_counter()
        for _ in range(reps):
            model.forward(slots.y, pe_np, slots.h_hat, slots.active, ones(B, U), num_it)
        return B * reps / (time.perf_counter() - t0)

    res = {}
    for tag, th in (("all", all_threads), ("1thread", 1)):
        _progress(f"cpu baseline, {th} threads")
        torch.set_num_threads(th)
        res[tag] = {"threads": th, "cfg1_b1_p50_ms": round(p50_b1(40 if th > 1 else 25), 3),
                    "cfg2_b128_slots_per_s": round(b128(2 if th > 1 else 1), 2)}
    torch.set_num_threads(torch_default)
    return {"value": res["all"]["cfg2_b128_slots_per_s"], "unit": "slots/s", "cores": all_threads,
            "threads": all_threads, "torch_default_threads": torch_default, "cgroup_cpu_quota": quota,
            "kind": "port",
            "sample": f"torch-CPU fp32 restatement (oracle/cgnn_torch.py), bench workload cfg2 "
                      f"({B} slots, {U} users, {args.prbs} PRB, num_it {num_it}) x2 batches at {all_threads} threads "
                      f"(value), plus cfg1 (1 UE, B=1) p50 latency and 1-thread runs",
            "cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count(),
            "affinity_cpus": affinity,
            "all_threads": res["all"], "one_thread": res["1thread"]}


if __name__ == "__main__":
    main()
