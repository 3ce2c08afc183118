"""Benchmark: depth maps/sec of the TransMVSNet hot path at DTU 864x1152, N=5, 48/32/8.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode replica|views] [--no-cpu-baseline]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Without a launcher, --gpus N > 1 makes this (GPU-untouched) process spawn N fresh rank processes
(rendezvous on 127.0.0.1, RCCL); under torchrun each process is one rank (WORLD_SIZE from the env).

A step is one hot-path forward (TransMVSNet.forward_features: FMT + pathway + 3-stage
stage glue / fused cost volume / CostRegNet / softmax-WTA) of one depth map from synthetic
FeatureNet-shaped features already resident in HBM; random-init weights of the reference
architecture (key-seeded, transmvsnet_amd.synthetic). FeatureNet (the next row)
is outside the timed step. Multi-GPU:
  replica (default) -- every rank computes its own depth maps, no collective ("weak");
  views             -- the 4 source views are sharded over ranks, one RCCL all-reduce of
                       (sum w*sim, sum w) per stage (transmvsnet_amd.distributed); with more
                       ranks than source views, replicas x view-shard groups (8 ranks: 2 x 4).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist

H, W, NVIEWS = 864, 1152, 5
NDEPTHS = (48, 32, 8)
C_STAGE = (32, 16, 8)
SCALES = (4, 2, 1)
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
PEAK_F32_MFMA_TFS = 157.3  # MI355X_MICROARCH.md: fp32 MFMA dense peak
# vector-memory address unit (TA) gather rate: 64 B/clk/CU (a 64-lane 16-B load costs >= 16 cycles,
# measured by scripts/micro/ta_mask.hip) x 256 CUs x 2.4 GHz
PEAK_TA_GBS = 64 * 256 * 2.4


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mode", choices=("replica", "views"), default="replica")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="nccl = RCCL (the product path); gloo only to rehearse the launcher with more ranks than GPUs")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads for cpu_baseline; 0 = the cores this process may run on")
    ap.add_argument("--cpu-runs", type=int, default=3, help="timed oracle runs (after 1 warm-up); median")
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--no-overlap", action="store_true", help="run the FMT pathway on the main stream (A/B)")
    ap.add_argument("--e2e-steps", type=int, default=10,
                    help="timed full forward() passes (images -> depth, FeatureNet included); 0 = skip")
    ap.add_argument("--side-priority", type=int, default=0,
                    help="stream priority of the FMT-pathway side stream (lower = higher; A/B knob)")
    ap.add_argument("--batch2-steps", type=int, default=10,
                    help="secondary line: B=2 per step (samples on two concurrent streams), 0 = skip")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch the step's kernels from Python every step instead of replaying one HIP graph")
    ap.add_argument("--train-steps", type=int, default=3,
                    help="timed C5 training steps of the DepthNet stages (transmvsnet_amd.train); 0 = skip")
    return ap.parse_args()


class EventTimer:
    """HIP events around every C-ABI launch, on the stream the kernels are launched on."""

    def __init__(self):
        self.spans = []

    def begin(self, name):
        if name == "tmvs_bn_fold":
            return None
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
        return (name, e0)

    def end(self, tok):
        if tok is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(torch.cuda.current_stream())
        self.spans.append((tok[0], tok[1], e1))

    def durations(self):
        torch.cuda.synchronize()
        return [(n, a.elapsed_time(b)) for n, a, b in self.spans]


def algorithmic():
    """Per-depth-map work units (SURVEY.md 8d / BASELINE.md 3)."""
    v = NVIEWS - 1
    warp_bytes, cr_flop = [], []
    for s in range(3):
        p = (H // SCALES[s]) * (W // SCALES[s])
        warp_bytes.append(4 * p * (C_STAGE[s] * (1 + v) + 2 * NDEPTHS[s] + v))
        cr_flop.append(6912 * NDEPTHS[s] * p)
    return warp_bytes, cr_flop


def gather_bytes():
    """Bilinear tap traffic of the warp per depth map through the vector L1 (SURVEY.md 8d companion
    bound): 16 * C * D * P * V bytes per stage (4 taps x C fp32 per pixel, plane and source view)."""
    v = NVIEWS - 1
    return [16 * C_STAGE[s] * NDEPTHS[s] * (H // SCALES[s]) * (W // SCALES[s]) * v for s in range(3)]


def make_inputs(device, seed_feat=2):
    from transmvsnet_amd import synthetic
    proj = synthetic.synthetic_cameras(NVIEWS, H, W, seed=1)
    dv = synthetic.synthetic_depth_values(1)
    return synthetic.stacked_features(NVIEWS, H, W, seed=seed_feat), proj, dv


def batch2_timing(model, feats, proj, dv_dev, steps, graphed):
    """Secondary line (NOT the headline, which is B=1): two depth maps per step -- the bench's sample
    twice, computed independently -- on two concurrent streams, as a server running requests side by side
    would: with graphs, one captured B=1 step per stream, both replayed per step (each graph with its own
    outputs); eagerly, one B=2 forward_features call (TransMVSNet.batch_streams)."""
    main = torch.cuda.current_stream()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    split = model.split_fmt
    if graphed:
        # two requests side by side: each graph's FMT in one stream (its side-stream fork measured slower next to
        # the other request's graph, profiles/r22/batch2_ab.txt); the B = 1 headline keeps the fork
        model.split_fmt = False
        graphs = []
        for st in streams:
            st.wait_stream(main)
            with torch.cuda.stream(st):
                for _ in range(2):
                    model.forward_features(feats, proj, dv_dev, (H, W))
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                model.forward_features(feats, proj, dv_dev, (H, W))
            graphs.append(g)
        torch.cuda.synchronize()
        model.split_fmt = split

        def step():
            ev = torch.cuda.Event()
            ev.record(main)
            for st, g in zip(streams, graphs):
                st.wait_event(ev)
                with torch.cuda.stream(st):
                    g.replay()
            for st in streams:
                main.wait_stream(st)
    else:
        f2 = {k: torch.cat([v, v], 0).contiguous() for k, v in feats.items()}
        p2 = {k: torch.cat([v, v], 0) for k, v in proj.items()}
        d2 = torch.cat([dv_dev, dv_dev], 0)

        def step():
            model.forward_features(f2, p2, d2, (H, W))
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"depth_maps_per_s": round(2 * steps / el, 3), "ms_per_step": round(el / steps * 1e3, 3), "steps": steps,
            "depth_maps_per_step": 2, "streams": 2,
            "launch": "one HIP graph per stream, replayed concurrently" if graphed else "eager B=2, one stream per sample",
            "note": "secondary: two depth maps per step on two concurrent streams; the headline value is one per step"}


def resolve_launch(gpus, env):
    """How this invocation maps onto ranks (no GPU call is made here).

    -> ("spawn", N): no launcher env and --gpus N > 1: this parent spawns N fresh rank processes;
       ("rank", world, rank, local_rank): run one rank (torchrun env, or a single process).
    """
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if gpus not in (1, world):
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}")
        return ("rank", world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", env.get("RANK", "0"))))
    if gpus > 1:
        return ("spawn", gpus)
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    return ("rank", 1, 0, 0)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank, world, port):
    """Environment of spawned rank `rank` (torchrun's variables, rendezvous on 127.0.0.1)."""
    return {"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_WORLD_SIZE": str(world),
            "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)}


def _spawned(rank, args, world, port):
    os.environ.update(rank_env(rank, world, port))
    run(args, world, rank, rank)


def main():
    args = _args()
    how = resolve_launch(args.gpus, os.environ)
    if how[0] == "spawn":
        # this parent has made no GPU call: start N fresh interpreters (spawn, not fork/exec of a
        # GPU-initialised process), one per GPU; a failing rank raises here
        import torch.multiprocessing as mp
        mp.start_processes(_spawned, args=(args, how[1], _free_port()), nprocs=how[1], join=True,
                           start_method="spawn")
        return
    _, world, rank, local = how
    run(args, world, rank, local)


def run(args, world, rank, local):
    ndev = torch.cuda.device_count()
    if local >= ndev and args.dist_backend == "nccl":
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local} but {ndev} are visible")
    local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != world:
            raise RuntimeError(f"process group has {dist.get_world_size()} ranks, expected {world}")

    from transmvsnet_amd import TransMVSNet, ops, synthetic
    model = TransMVSNet().eval()
    model.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(model), seed=0, sharpen=100.0))
    model = model.to(dev)
    model.overlap_pathway = not args.no_overlap
    model.side_priority = args.side_priority
    feats_cpu, proj, dv = make_inputs(dev)
    feats = {k: v.to(dev) for k, v in feats_cpu.items()}
    dv_dev = dv.to(dev)
    shard = None
    if args.mode == "views" and world > 1:
        # replica x view-shard groups: more ranks than source views run several view-sharded groups
        from transmvsnet_amd.distributed import make_view_shard
        shard = make_view_shard(rank, world, NVIEWS - 1)

    def step():
        return model.forward_features(feats, proj, dv_dev, (H, W), view_shard=shard)

    eager_step = step
    # a view-sharded step replays as one graph too: RCCL all-reduces are captured on the step's stream
    # (gloo's CPU-side collectives cannot be captured)
    graphed = not args.no_graph and (shard is None or args.dist_backend == "nccl")
    with torch.no_grad():
        for _ in range(args.warmup):
            out = step()
        torch.cuda.synchronize()
        if graphed:
            # one HIP graph of the whole step (every kernel of FMT, pathway side stream, 3 stages),
            # captured after the warm-up and replayed per step: the same kernels on the same resident
            # inputs, without the host's per-launch cost (a slow or busy host otherwise stretched the
            # 3.8 ms step to 6.8 ms, profiles/r10p)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                g_out = step()
            torch.cuda.synchronize()

            def step():  # noqa: F811
                graph.replay()
                return g_out
            out = step()
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        elapsed = t1 - t0
        ranks_ok = None
        if world > 1:
            t = torch.tensor([elapsed], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            # every rank ran the same K steps on the same inputs: its final depth map must be
            # bitwise identical to every other rank's (deterministic kernels), else the job failed
            chk = torch.tensor([float(args.steps), float(out["depth"].double().sum())], device=dev, dtype=torch.float64)
            allc = [torch.empty_like(chk) for _ in range(world)]
            dist.all_gather(allc, chk)
            allc = [c.cpu().tolist() for c in allc]
            if any(c != allc[0] for c in allc):
                raise RuntimeError(f"ranks disagree (steps, depth checksum): {allc}")
            ranks_ok = {"ranks": world, "steps_each": args.steps, "depth_checksum": allc[0][1]}

        eager = None
        if graphed:
            # the same K steps launched eagerly from Python, outside the timed region: the form a caller
            # with per-sample cameras runs (the proj rows are kernel arguments frozen in the captured graph)
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            te = time.perf_counter()
            for _ in range(args.steps):
                eager_step()
            torch.cuda.synchronize()
            el = time.perf_counter() - te
            if world > 1:
                t = torch.tensor([el], device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el = float(t.item())
            mps = shard.replicas if shard is not None else (1 if args.mode == "views" else world)
            eager = {"ms_per_step": round(el / args.steps * 1e3, 3),
                     "depth_maps_per_s": round(mps * args.steps / el, 3), "steps": args.steps,
                     "launch": "eager (one Python call per C-ABI entry point per step; not the headline)"}

        # instrumented steps (outside the timed region): per-launch HIP-event durations
        timer = EventTimer()
        model.decomposed = True   # same kernels, one C-ABI call each, so each gets its own event pair
        ops.set_timer(timer)
        if shard is not None:
            shard.timer = timer
        for _ in range(args.profile_steps):
            eager_step()
        ops.set_timer(None)
        if shard is not None:
            shard.timer = None
        model.decomposed = False
        spans = timer.durations()
        # the same instrumentation on the timed step's own form (fused stage calls, pathway on its side
        # stream concurrently with stage 1): per-call durations as they overlap in the timed region
        otimer = EventTimer()
        ops.set_timer(otimer)
        for _ in range(args.profile_steps):
            eager_step()
        ops.set_timer(None)
        ospans = otimer.durations()

        coherent = coherent_warp_timing(model, feats, proj, dv_dev) if args.profile_steps > 0 and shard is None else None
        e2e = end_to_end(model, args.e2e_steps, proj, dv_dev, dev) if args.e2e_steps > 0 and shard is None else None
        batch2 = (batch2_timing(model, feats, proj, dv_dev, args.batch2_steps, graphed)
                  if args.batch2_steps > 0 and shard is None else None)
    train = (train_timing(args.train_steps, dev, world, use_graph=not args.no_graph)
             if args.train_steps > 0 and shard is None else None)

    maps_per_step = shard.replicas if shard is not None else (1 if args.mode == "views" else world)
    value = maps_per_step * args.steps / elapsed
    per_kernel = {}
    for n, ms in spans:
        per_kernel.setdefault(n, []).append(ms)
    steps_p = max(1, args.profile_steps)
    breakdown = {n: round(sum(v) / steps_p, 4) for n, v in per_kernel.items()}
    overlapped = {}
    for n, ms in ospans:
        overlapped[n] = overlapped.get(n, 0.0) + ms / steps_p
    overlapped = {n: round(v, 4) for n, v in overlapped.items()}

    warp_bytes, cr_flop = algorithmic()
    warp_ms = per_kernel.get("tmvs_warp_corr", [])
    cr_ms = per_kernel.get("tmvs_costregnet", [])
    kern = []
    if warp_ms:
        per_launch = np.array(warp_ms).reshape(steps_p, -1).mean(0)  # stage order
        ach = sum(warp_bytes) / (per_launch.sum() * 1e-3) / 1e9
        kern.append({"kernel": "tmvs_warp_corr", "bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": None,
                     "ms_per_depth_map": round(float(per_launch.sum()), 4),
                     "avg_launch_us": round(float(per_launch.mean()) * 1e3, 2), "launches_per_depth_map": 3,
                     "per": "depth map (3 launches: stages 1-3); achieved = algorithmic bytes / summed duration",
                     "algorithmic_bytes": int(sum(warp_bytes)),
                     "per_stage_ms": [round(float(x), 4) for x in per_launch]})
    if warp_ms:  # the same launches against the address-unit bound that actually limits them
        per_launch = np.array(warp_ms).reshape(steps_p, -1).mean(0)
        gb = gather_bytes()
        ach = sum(gb) / (per_launch.sum() * 1e-3) / 1e9
        kern.append({"kernel": "tmvs_warp_corr (gather)", "bound": "ta", "achieved": round(ach, 1), "peak": PEAK_TA_GBS,
                     "unit": "GB/s", "frac": round(ach / PEAK_TA_GBS, 4), "traffic": None,
                     "ms_per_depth_map": round(float(per_launch.sum()), 4),
                     "per": "depth map; achieved = bilinear tap bytes 16*C*D*P*V / summed duration; peak = the "
                            "measured 64 B/clk/CU address-unit rate x 256 CUs x 2.4 GHz",
                     "gather_bytes": int(sum(gb)),
                     "per_stage_frac": [round(b / (t * 1e-3) / 1e9 / PEAK_TA_GBS, 3) for b, t in zip(gb, per_launch)]})
    if cr_ms:
        per_launch = np.array(cr_ms).reshape(steps_p, -1).mean(0)
        ach = sum(cr_flop) / (per_launch.sum() * 1e-3) / 1e12
        kern.append({"kernel": "tmvs_costregnet", "bound": "mfma", "achieved": round(ach, 2),
                     "peak": PEAK_F32_MFMA_TFS, "unit": "TFLOP/s", "frac": round(ach / PEAK_F32_MFMA_TFS, 4),
                     "traffic": None, "ms_per_depth_map": round(float(per_launch.sum()), 4),
                     "per": "depth map (3 tmvs_costregnet_wta calls: 11 CostRegNet kernels each, the prob conv fused with softmax/WTA at stages 2/3, + the softmax kernel at stage 1)",
                     "algorithmic_flop": int(sum(cr_flop)),
                     "per_stage_ms": [round(float(x), 4) for x in per_launch]})
    if coherent is not None:
        kern.append(coherent)
    # headline roofline: the north-star kernel (warp_corr_kernel, one launch per stage; its
    # rocprofv3 average over the 3 launches of a step is avg_launch_us); CostRegNet (11
    # kernels per stage) is listed beside it in roofline_kernels
    dominant = next((k for k in kern if k["kernel"] == "tmvs_warp_corr"), None) or (kern[0] if kern else None)
    pmc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc))
            src = traffic.get("_meta", {}).get("source", "profiles/pmc_traffic.json")
            for k in kern:
                if k["kernel"] in traffic:
                    # NOT measured in this run: rocprofv3 PMC passes of an earlier round (provenance below)
                    k["traffic"] = traffic[k["kernel"]]
                    k["traffic_source"] = f"profiles/pmc_traffic.json: {src}"
        except Exception:
            pass

    comm = None
    if shard is not None:
        ar = per_kernel.get("rccl_all_reduce", [])
        if ar:
            per_launch = np.array(ar).reshape(steps_p, -1).mean(0)
            comm = {"collective": "all_reduce(SUM) of packed [D+1,h,w] fp32 per stage",
                    "bytes_per_stage": shard.comm_bytes[:3], "ms_per_stage": [round(float(x), 4) for x in per_launch],
                    "busbw_GBs": [round(2 * (world - 1) / world * b / (ms * 1e-3) / 1e9, 1)
                                  for b, ms in zip(shard.comm_bytes[:3], per_launch)]}
    cpu = None
    l1 = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, l1 = cpu_baseline(args.cpu_threads, args.cpu_runs, feats_cpu, proj, dv, out)

    if rank == 0:
        line = {
            "metric": "depth maps/sec @ DTU 864x1152 N=5 (48/32/8 hyp); Abs depth L1 vs ref",
            "value": round(value, 3),
            "unit": "depth_maps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "replica" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded FeatureNet-shaped features, DTU-like cameras, key-seeded random weights)",
            "config": {"workload": "DTU 864x1152, N=5 views, cascade 48/32/8, B=1, hot path from FeatureNet "
                                   "outputs (FMT+pathway+stage glue+cost volume+CostRegNet+softmax/WTA)",
                       "global_batch": maps_per_step, "parallelism": f"{args.mode}{world}",
                       "launch": "hip_graph replay" if graphed else "eager"},
            "eager": eager,
            "roofline": dominant,
            "roofline_kernels": kern,
            "kernel_ms_per_depth_map": breakdown,
            "kernel_ms_source": "HIP events per C-ABI call in a DECOMPOSED pass (one call per op, pathway overlap "
                                "off; roofline_kernels use it); call_ms_overlapped = the timed step's own calls "
                                "(fused tmvs_depth_stage at stages 2/3, pathway on its side stream)",
            "call_ms_overlapped": overlapped,
            "cpu_baseline": cpu,
            "abs_depth_l1_vs_ref": l1,
            "end_to_end": e2e,
            "batch2_concurrent": batch2,
            "train_depth_stages": train,
        }
        if ranks_ok is not None:
            line["ranks_check"] = ranks_ok
        if comm is not None:
            line["allreduce"] = comm
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def coherent_warp_timing(model, feats, proj, dv_dev, reps=20):
    """Secondary workload (roofline_kernels, not the headline): the stage-2/3 cost-volume launches
    (tmvs_warp_corr) on COHERENT hypotheses next to the bench's own. The bench's random features make its
    stage-1/2 WTA depth -- which the stage-2/3 hypotheses are built from (models/TransMVSNet.py:174-190) --
    spatially incoherent, so neighbouring pixels' bilinear taps land in unrelated source neighbourhoods;
    real scenes give smooth depth. Same stage features, cameras, view weights and kernels, with the
    hypotheses built by tmvs_stage_hypotheses from a slanted plane 600 + 150 x/W + 100 y/H mm instead of the
    GPU's own previous-stage depth. Per stage: HIP-event median of `reps` launches; tap bytes 16 C D P V over
    the address unit's rate, algorithmic HBM bytes over 8 TB/s."""
    from transmvsnet_amd import ops
    from transmvsnet_amd.model import STAGE_SCALES
    dev = dv_dev.device
    with torch.no_grad():
        out, vw = model.forward_features(feats, proj, dv_dev, (H, W), return_view_weights=True)
        prep = model._prepared(dev)
        s1, s2, s3 = feats["stage1"][0], feats["stage2"][0], feats["stage3"][0]
        n, _, h1, w1 = s1.shape
        st1 = model._fmt(s1, prep).view(n, h1, w1, 32)
        st2 = ops.fmt_pathway(st1, s2, prep["red1"], prep["sm1"])
        fs = (st1, st2, ops.fmt_pathway(st2, s3, prep["red2"], prep["sm2"]))
        rows = {k: ops.proj_rows(proj[k]) for k in ("stage2", "stage3")}
        per = {}
        for s in (1, 2):
            name = f"stage{s + 1}"
            hp, wp = H // STAGE_SCALES[s - 1], W // STAGE_SCALES[s - 1]
            yy, xx = torch.meshgrid(torch.arange(hp, dtype=torch.float32), torch.arange(wp, dtype=torch.float32),
                                    indexing="ij")
            plane = (600.0 + 150.0 * xx / wp + 100.0 * yy / hp)[None].to(dev).contiguous()
            hyps = {"bench": out[name]["depth_values"].contiguous(),
                    "coherent": ops.stage_hypotheses(dv_dev[0:1], plane, model.ndepths[s], model.depth_interals_ratio[s],
                                                     (H, W), STAGE_SCALES[s])}
            f = fs[s]
            _, h, w, c = f.shape
            d, v, p = model.ndepths[s], NVIEWS - 1, h * w
            tap, alg = 16 * c * d * p * v, 4 * p * (c * (1 + v) + 2 * d + v)
            row = {}
            for kind, hyp in hyps.items():
                for _ in range(3):
                    ops.warp_corr(f[0:1], f[1:].unsqueeze(0), rows[name], hyp, view_w_in=vw, vw_shift=s)
                ts = []
                for _ in range(reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    ops.warp_corr(f[0:1], f[1:].unsqueeze(0), rows[name], hyp, view_w_in=vw, vw_shift=s)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                us = float(np.median(ts))
                row[kind] = {"us": round(us, 2), "ta_frac": round(tap / (us * 1e-6) / 1e9 / PEAK_TA_GBS, 4),
                             "hbm_frac": round(alg / (us * 1e-6) / 1e9 / PEAK_HBM_GBS, 4)}
            per[name] = row
    us = sum(per[k]["coherent"]["us"] for k in per)
    tap = sum(gather_bytes()[1:])
    return {"kernel": "tmvs_warp_corr (gather, coherent stage-2/3 hypotheses)", "bound": "ta",
            "achieved": round(tap / (us * 1e-6) / 1e9, 1), "peak": PEAK_TA_GBS, "unit": "GB/s",
            "frac": round(tap / (us * 1e-6) / 1e9 / PEAK_TA_GBS, 4), "traffic": None,
            "per": "stages 2+3 of one depth map, one launch each (HIP events, median of %d); secondary workload: "
                   "hypotheses from a slanted plane (600 + 150 x/W + 100 y/H mm) instead of the bench's incoherent "
                   "WTA depth" % reps,
            "per_stage": per}


def end_to_end(model, steps, proj, dv_dev, dev):
    """The whole TransMVSNet.forward (images -> depth, FeatureNet + DCN included) beside the hot-path
    step: synthetic U[0,1) images [1,N,3,H,W] resident in HBM, HIP events on the current stream,
    median of `steps` after 2 warm-ups. FeatureNet alone is timed the same way."""
    from transmvsnet_amd import synthetic
    imgs = synthetic.synthetic_images(NVIEWS, H, W).to(dev)

    def timed(fn):
        ts = []
        for i in range(steps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    t_all = timed(lambda: model.forward(imgs, proj, dv_dev))
    t_feat = timed(lambda: model.feature(imgs.reshape(NVIEWS, 3, H, W)))
    return {"depth_maps_per_s": round(1e3 / t_all, 3), "ms_per_depth_map": round(t_all, 3),
            "featurenet_ms": round(t_feat, 3), "steps": steps,
            "workload": "TransMVSNet.forward(imgs [1,5,3,864,1152], proj, depth_values): FeatureNet (HIP: "
                        "tmvs_conv2d_bn_relu trunk, tmvs_fpn_merge, tmvs_conv3x3_nhwc, tmvs_dcn_fused) + the hot "
                        "path above"}


def _train_setup(dev):
    from transmvsnet_amd import TransMVSNet, loss as hip_loss, synthetic
    from transmvsnet_amd.train import FlatAdam, depth_stages_train, fmt_train, pathway_train
    h5, w5, n5 = 576, 768, 4
    m = TransMVSNet()
    m.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(m), seed=0, sharpen=100.0))
    m = m.to(dev)
    imgs = synthetic.synthetic_images(n5, h5, w5, seed=8).to(dev)
    feats = synthetic.stacked_features(n5, h5, w5, seed=5)
    leaves = {"stage1": feats["stage1"][0].contiguous().to(dev).requires_grad_(),
              "stage2": feats["stage2"][0].contiguous().to(dev).requires_grad_(),
              "stage3": feats["stage3"][0].contiguous().to(dev).requires_grad_()}
    proj = synthetic.synthetic_cameras(n5, h5, w5, seed=6)
    dv = synthetic.synthetic_depth_values(1).to(dev)
    g = torch.Generator().manual_seed(7)
    gt = {f"stage{s + 1}": (425.0 + 500.0 * torch.rand(1, h5 >> (2 - s), w5 >> (2 - s), generator=g)).to(dev)
          for s in range(3)}
    mask = {k: torch.ones_like(v) for k, v in gt.items()}
    dint = float(dv[0, 1] - dv[0, 0])  # the sample's depth_interval (finetune.py:159)
    interval = torch.tensor([dint])  # host: focal_loss_bld reads it as a number (no device sync in the step)
    opt = FlatAdam(list(m.parameters()), lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4)  # finetune.py:27,29,324

    def full_step():
        m.train()
        opt.zero_grad()
        outputs = m(imgs, proj, dv)
        loss = hip_loss.focal_loss_bld(outputs, gt, mask, interval, dlossw=[1.0, 1.0, 1.0])[0]
        loss.backward()
        opt.allreduce()
        opt.step()

    def features_step():
        for p in leaves.values():
            p.grad = None
        opt.zero_grad()
        st1 = fmt_train(m, leaves["stage1"])
        st2, st3 = pathway_train(m, st1, leaves["stage2"], leaves["stage3"])
        depth_stages_train(m, {"stage1": st1, "stage2": st2, "stage3": st3}, proj, dv, gt, mask, (h5, w5),
                           dlossw=(1.0, 1.0, 1.0), loss="focal_bld", depth_interval=dint)
        opt.allreduce()
        opt.step()

    return full_step, features_step, m


def train_steps(dev):
    """The C5 training closures (full_step, features_step, model) train_timing times (also run alone
    by scripts/diag/train_prof.py under rocprofv3)."""
    return _train_setup(dev)


def train_timing(steps, dev, world, use_graph=True):
    """C5 training step (BlendedMVS 768x576, N=4, 48/32/8, one sample per rank): the reference's
    train_sample body (finetune.py:144-168) on the drop-in model -- model.train(); zero_grad;
    outputs = model(imgs, proj, depth_values) (FeatureNet + DCN, FMT, pathway, 3 DepthNet stages, all
    HIP with autograd); focal_loss_bld (dlossw 1,1,1) -> loss.backward() (HIP backward of every block,
    FeatureNet/DCN included); DDP's gradient all-reduce when world > 1; Adam step (FlatAdam). HIP
    events, median of `steps` after 1 warm-up; max over ranks. Also times the same step from
    FeatureNet's outputs (the round-2 measurement, for continuity)."""
    full_step, features_step, m = _train_setup(dev)

    def timed(fn):
        ts = []
        for i in range(steps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if i > 0:
                ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        if world > 1:
            t = torch.tensor([ms], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ms = float(t.item())
        return ms

    def graphed(fn):
        """fn captured as one HIP graph (forward, autograd backward, gradient gather, Adam with its step
        counter on the device; the warp backwards' overflow flags are checked after the replays) and
        replayed; None when the capture fails (then the step is timed eagerly)."""
        if world > 1 or not use_graph:
            return None
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                fn()
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize()
            g = _train.TrainStepGraph(fn, m)  # per-graph overflow flags; replay() re-keys the inference caches
            torch.cuda.synchronize()
            graphs.append(g)
            return g.replay
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line, the eager timing stands
            launch_notes.append(f"{getattr(fn, '__name__', 'step')}: capture failed ({type(e).__name__}: {str(e)[:120]})")
            torch.cuda.synchronize()
            return None

    from transmvsnet_amd import train as _train
    launch_notes, graphs = [], []
    ms_eager = timed(full_step)
    ms_feat_eager = timed(features_step)
    g_full, g_feat = graphed(full_step), graphed(features_step)
    ms = timed(g_full) if g_full else ms_eager
    ms_feat = timed(g_feat) if g_feat else ms_feat_eager
    for g in graphs:
        g.check_flags()
    nbytes = sum(p.numel() for p in m.parameters()) * 4
    return {"ms_per_sample": round(ms, 3), "samples_per_s": round(world * 1e3 / ms, 3), "ranks": world,
            "grad_allreduce_bytes": nbytes if world > 1 else 0,
            "ms_per_sample_from_features": round(ms_feat, 3),
            "launch": ("hip_graph replay" if g_full else "eager") + "; eager: "
                      f"{round(ms_eager, 3)} / {round(ms_feat_eager, 3)} ms" + (f"; {'; '.join(launch_notes)}" if launch_notes else ""),
            "workload": "BlendedMVS 768x576, N=4, 48/32/8, 1 sample per rank: finetune.py:144-168's train_sample "
                        "body on the drop-in model -- model.train(); optimizer.zero_grad(); outputs = model(imgs, "
                        "proj, depth_values); focal_loss_bld(..., dlossw 1,1,1); loss.backward(); optimizer.step() -- "
                        "forward + backward on HIP of FeatureNet (trunk convs, FPN merges, DCNs: offset/mask conv + "
                        "deformable conv), the FMT (8 encoder layers), FMT_with_pathway's lateral steps and the "
                        "DepthNet stages (per-view cost volumes, view aggregation + train-mode PixelwiseNet, "
                        "CostRegNet, softmax/WTA, loss + d/dlogits), DDP gradient all-reduce (one flat buffer) + "
                        "Adam (tmvs_adam_step). ms_per_sample_from_features: the same step from FeatureNet's outputs "
                        "(FeatureNet excluded; round 2's measurement)"}


def host_cores():
    """(cores this process may run on, cgroup CPU quota or None, CPU model)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return n, quota, model


def parity_report(gpu_out, ref, sref):
    """Abs depth L1 vs the reference restatement, per stage, every differing pixel classified by
    oracle/parity.py -- the classifier tests/test_gpu_fullsize.py asserts with: near ties (reference top-2
    log-prob margin < 1e-4); in the plain cascade, flips inside CostRegNet's receptive-field
    footprint of hypotheses moved by an upstream near-tie flip; and stages 2/3 against the reference
    cascade continued from the GPU's own previous-stage depths (sref: identical hypotheses, the near-tie
    rule alone). other_flips counts what none of these explains (a real mismatch)."""
    from oracle import parity
    casc = parity.cascade_report(gpu_out, ref)
    seeded = parity.gpu_seeded_report(gpu_out, sref)
    keep = ("mean_abs_mm", "max_abs_mm", "differing", "near_tie_flips", "cascade_explained", "other_flips",
            "max_flip_margin", "moved_hypotheses", "logprob_spread")
    rep = {}
    for s in (1, 2, 3):
        rep[f"stage{s}"] = {k: v for k, v in casc[f"cascade_stage{s}"].items() if k in keep}
        if s > 1:
            rep[f"stage{s}"]["gpu_seeded"] = {k: v for k, v in seeded[f"gpu_seeded_stage{s}"].items() if k in keep}
    d3 = rep["stage3"]
    return {"stage3_mean_abs_mm": d3["mean_abs_mm"], "stage3_max_abs_mm": d3["max_abs_mm"],
            "stage3_frac_pixels_differing": d3["differing"] / gpu_out["depth"].numel(),
            "stage3_gpu_seeded_mean_abs_mm": d3["gpu_seeded"]["mean_abs_mm"],
            "other_flips": sum(rep[f"stage{s}"]["other_flips"] for s in (1, 2, 3))
            + sum(rep[f"stage{s}"]["gpu_seeded"]["other_flips"] for s in (2, 3)),
            "per_stage": rep, "near_tie_margin": parity.MARGIN,
            "classifier": "oracle/parity.py (the tests' classifier): near tie < 1e-4; cascade = CostRegNet receptive "
                          "field (40 px) around moved hypotheses; gpu_seeded = reference stages 2/3 from the GPU's "
                          "previous-stage depth"}


def cpu_baseline(threads, runs, feats_cpu, proj, dv, gpu_out):
    """The oracle (torch-CPU restatement of the reference forward) on the host cores.

    SURVEY.md 8d recipe: torch threads = the cores this process may run on (sched_getaffinity,
    capped by a cgroup CPU quota when one is set), 1 untimed warm-up run, then `runs` timed runs of
    one full DTU depth map (same inputs/weights as the GPU step); the median is reported. Also
    returns the per-stage 'Abs depth L1 vs ref' of the GPU step against the last run's output.
    """
    from oracle import parity
    from oracle import transmvs_ref as oracle
    from transmvsnet_amd import TransMVSNet, synthetic
    n_aff, quota, cpu_model = host_cores()
    if threads <= 0:
        threads = n_aff if quota is None else max(1, min(n_aff, int(quota)))
    torch.set_num_threads(threads)
    shapes = synthetic.state_dict_shapes(TransMVSNet())
    sd = synthetic.synthetic_state_dict(shapes, seed=0, sharpen=100.0)
    feats = [{k: v[:, i] for k, v in feats_cpu.items()} for i in range(NVIEWS)]
    ts = []
    with torch.no_grad():
        for i in range(runs + 1):
            t0 = time.perf_counter()
            ref = oracle.forward_from_features(sd, feats, proj, dv, (H, W))
            t1 = time.perf_counter()
            if i > 0:
                ts.append(t1 - t0)
        sref = oracle.forward_from_features(sd, feats, proj, dv, (H, W), seed_depth=parity.seed_depths(gpu_out))
    med = float(np.median(ts))
    quota_txt = f", cgroup quota {quota:g} CPUs" if quota is not None else ""
    return ({"value": round(1.0 / med, 5), "unit": "depth_maps/s", "cores": threads, "kind": "port",
             "sample": f"1 DTU depth map (864x1152, N=5, 48/32/8) through the oracle's hot path (torch-CPU fp32); "
                       f"median of {runs} timed runs after 1 warm-up: {med:.2f} s (runs {', '.join(f'{t:.2f}' for t in ts)}); "
                       f"{threads} threads = sched_getaffinity {n_aff}{quota_txt}; {cpu_model}"},
            parity_report(gpu_out, ref, sref))


if __name__ == "__main__":
    main()
