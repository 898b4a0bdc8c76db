"""bench.py — train-step throughput of the MI355X NeuS hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|...] [--graph]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
    python bench.py --gpus 2 --dry --backend gloo      (launcher check on the CPU, no HIP work)

Without WORLD_SIZE in the environment, `--gpus N > 1` starts the N rank processes itself (one per
GPU, before any GPU call); under a launcher WORLD_SIZE must equal --gpus.

Metric (BASELINE.json): rays/sec of a full training step incl. backward at
4096 rays x 128 samples per GPU (64 coarse + 4x16 importance, fp32, fixed
poses, synthetic data): patch sampling + ray generation, the HIP renderer
forward, L1 rgb + 0.1 eikonal + edge-aware / plain depth smoothness, the HIP
backward (incl. the ∇ₓSDF double backward), the gradient all-reduce (N > 1)
and Adam.  Weak scaling: every rank renders its own 4096 rays.  The timed
steps run uninstrumented.

The JSON line also carries
  roofline      the dominant kernel (the cn_linear / cn_wgrad launch class with the
                most time), from a separate instrumented pass after the timed steps
                (HIP events around each launch on the launching stream):
                its algorithmic FLOPs and bytes per launch against the binding
                ceiling, max(FLOPs / MFMA peak of the GEMM mode, bytes / HBM
                peak); the kernel's duration is the rocprofv3 average of a committed
                kernel-stats CSV recorded for this very library build (its
                _lib_stamp.txt equals the loaded .so's stamp), else this run's HIP
                events (`frac_source` says which); `traffic` is the rocprofv3 PMC
                (FETCH_SIZE + WRITE_SIZE) per launch read from profiles/ when a
                counter pass for this kernel is committed;
  cpu_baseline  the CPU oracle (oracle/neus_oracle.py, a torch restatement of the
                reference path pinned to the reference's outputs) timed on this
                box's host cores: median of 5 steps at 1024 rays after a
                warm-up (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import datetime
import glob
import json
import os
import sys
import time
import warnings

import torch
import torch.distributed as dist

# no autograd graph may outlive a step (GraphedTrainer keeps none): an eager step after a captured one
# that warns about the AccumulateGrad node's stream would run under extra stream synchronisation
warnings.filterwarnings("error", message="The AccumulateGrad node's stream")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, = fp32 vector peak
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 (v_mfma_f32_32x32x16_bf16, 32 cycles)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E
# fp32-GEMM FLOP/s ceiling of each operand mode: bf16x6 issues six bf16 MFMAs per fp32 product
MODE_PEAK_TFLOPS = {"fp32": FP32_MFMA_PEAK_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS,
                    "bf16x6": BF16_MFMA_PEAK_TFLOPS / 6.0}
MODE_TEXT = {"fp32": "exact fp32 MFMA products (v_mfma_f32_32x32x2_f32)",
             "bf16x6": "fp32 GEMMs on the bf16 MFMA: both operands split into three bf16 terms, six products, "
                       "fp32 accumulate (error vs float64 <= the exact fp32 MFMA's; tests/test_gpu_x6.py)",
             "bf16": "bf16 MFMA operands (reduced precision), fp32 accumulate / activations"}
RAYS = 4096
SAMPLES = 128
GFLOP_PER_RAY_REF = 1.4809  # reference GEMM FLOPs per ray per train step (64+4x16)


def lib_stamp():
    """Digest of the sources, headers and flags the loaded libcopenerf.so was built from (the
    `.stamp` build() writes beside it), or None."""
    from copenerf import _lib
    try:
        with open(_lib.LIB_PATH + ".stamp") as f:
            return f.read().strip() or None
    except OSError:
        return None


def stats_stamp(csv_path):
    """The library stamp tools/profile_round.sh recorded beside a kernel-stats CSV, or None."""
    try:
        with open(csv_path.replace("_kernel_stats.csv", "_lib_stamp.txt")) as f:
            return f.read().strip() or None
    except OSError:
        return None


def rocprof_launch_ns(symbol, config, stamp):
    """Average duration (ns) of `symbol` in the newest committed rocprofv3 kernel-stats summary of
    this config's bench (profiles/<tag>_kernel_stats.csv for c2, <tag>_<config>_kernel_stats.csv
    otherwise) that was recorded for this very library build (its `_lib_stamp.txt` equals `stamp`),
    and the file; (None, None) otherwise."""
    import csv
    if not stamp:
        return None, None
    pat = "*_kernel_stats.csv" if config == "c2" else f"*_{config}_kernel_stats.csv"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pat)))
    if config == "c2":  # (another config's files carry its name before the suffix)
        files = [f for f in files if not any(f.endswith(f"_{c}_kernel_stats.csv") for c in CONFIGS if c != "c2")]
    files = [f for f in files if stats_stamp(f) == stamp]
    for f in reversed(files):
        try:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if row.get("Name") == symbol:
                        return float(row["AverageNs"]), os.path.relpath(f, ROOT)
        except (OSError, ValueError, KeyError):
            continue
    return None, None


def pmc_traffic(symbol, stamp=None):
    """Per-launch HBM bytes of `symbol` from the newest committed counter pass of this library build
    (tools/pmc_round.sh writes the build's stamp beside the pass: profiles/<tag>_pmc.json with
    <tag>_lib_stamp.txt)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")))
    for f in reversed(files):
        st = f[:-len("pmc.json")] + "lib_stamp.txt"
        try:
            if stamp is None or open(st).read().strip() != stamp:
                continue
        except OSError:
            continue
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(symbol)
        if k and k.get("hbm_bytes_per_launch"):
            return float(k["hbm_bytes_per_launch"]), os.path.relpath(f, ROOT)
    return None, None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _available_cpus():
    """The cores this process may run on (BASELINE.md's CPU-baseline plan): its affinity
    mask, capped by the cgroup CPU quota when one is set (a GPU box's share of a larger
    host: the affinity mask there lists every core of the machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(rays=1024, steps=5):
    """Time the CPU oracle (torch restatement of the reference path) on the host:
    one warm-up step, then the median of `steps` steps at `rays` rays (BASELINE.md's
    CPU-baseline plan)."""
    import statistics
    from tests.helpers import build_modules, oracle_params
    from oracle import neus_oracle as O
    threads = int(os.environ.get("COPENERF_CPU_THREADS", _available_cpus()))
    torch.set_num_threads(threads)
    mods = build_modules(678)
    g = torch.Generator().manual_seed(0)

    def one(R):
        P, Pc, var, leaves = oracle_params(*mods)
        o = torch.zeros(R, 3)
        d = torch.cat([(torch.rand(R, 2, generator=g) - 0.5), -torch.ones(R, 1)], -1)
        nrm = d.norm(dim=-1, keepdim=True)
        t0 = time.perf_counter()
        out = O.render(P, Pc, var, o, d / nrm, nrm, torch.zeros(1), torch.full((R, 1), 0.01), torch.full((R, 1), 5.0),
                       car=0.5, t_rand=torch.rand(R, 64, generator=g))
        loss = O.train_loss(out, torch.rand(R, 3, generator=g))
        torch.autograd.grad(loss, list(leaves.values()))
        return time.perf_counter() - t0

    one(rays)  # warm the allocator / MKL at the measured size
    times = [one(rays) for _ in range(steps)]
    med = statistics.median(times)
    return {"value": round(rays / med, 3), "unit": "rays/s", "cores": threads, "kind": "port",
            "sample": f"oracle/neus_oracle.py train step (fwd + L1/eikonal/smoothness loss + backward, no optimiser), "
                      f"{rays} rays x 128 samples (64+4x16), full-width nets, fp32, torch {torch.__version__} CPU, "
                      f"{threads} threads on '{_cpu_model()}'; median of {steps} steps after 1 warm-up "
                      f"(min {min(times):.2f} s, max {max(times):.2f} s per step)"}


C3_TRAIN = dict(sdf_consistency_enable_pose_grad=True, rgb_weight=0.33333, end_sdf_weight_increase_iteration=-1)
CONFIGS = {
    # name: (rays per GPU, trainer kwargs, workload text)
    "c2": (4096, {"mfma_dtype": "bf16x6"},
           "C2: synthetic scene, 4096 rays x 128 samples (64 coarse + 4x16 importance) per GPU, fp32, "
           "fixed poses, full train step (fwd + losses + bwd + Adam)"),
    "c2fp32": (4096, {"mfma_dtype": "fp32"}, "C2 with the exact-product fp32 MFMA GEMMs"),
    # C3 = Co3D/skateboard.yaml's pose optimisation: stage 1 (epochs < start_query_world_epoch),
    # where the camera motion is learned as the MotionNetwork jointly with the fields through the
    # scene-flow SDF loss, the flow-RGB warp and the SDF consistency at the world camera
    # (train.py:467-517); skateboard's options: sdf_consistency_enable_pose_grad, rgb_weight
    # 0.33333, a fixed sdf_weight (end_sdf_weight_increase_iteration -1)
    "c3": (4096, {"stage1": True, "mfma_dtype": "bf16", "start_it": 30000, "train_cfg": dict(C3_TRAIN)},
           "C3: Co3D/skateboard stage 1 on a synthetic 10-frame scene, 4096 rays x 128 samples per GPU, bf16 MLP "
           "MFMA (fp32 accumulate): MotionNetwork pose optimisation through the scene-flow SDF loss, flow-RGB warp "
           "to the 3 next frames and SDF consistency at the world camera with pose gradient"),
    "c3fp32": (4096, {"stage1": True, "mfma_dtype": "bf16x6", "start_it": 30000, "train_cfg": dict(C3_TRAIN)},
               "C3 as c3 with fp32 GEMMs (bf16x6)"),
    # stage 2 with pose refinement: rays from learnable SE(3) poses (PoseRetriever) in canonical
    # space, ray gradients into r, t (train.py:425-431; freeze_camera_pose_period finite)
    "c3pose": (4096, {"joint_pose": True, "mfma_dtype": "bf16x6", "start_it": 30000},
               "stage 2 with pose refinement: synthetic 10-frame scene, 4096 rays x 128 samples per GPU, fp32 "
               "(bf16x6), query in canonical space with learnable SE(3) camera poses (ray gradients)"),
    "infer": (518400, {"infer": True, "mfma_dtype": "bf16x6"},
              "inference: full 540x960 image (518,400 rays x 128 samples, eval mode, no jitter), forward only "
              "(sampler + SDF + ∇SDF + colour + compositing), 65,536-ray chunks, fp32"),
    "c2bf16": (4096, {"mfma_dtype": "bf16"},
               "C2 workload (4096 rays x 128 samples, fixed poses) with bf16 MLP MFMA (fp32 accumulate)"),
    # C4 = Co3D/skateboard (its stage-1 pose optimisation, as c3fp32) at 8192 rays per GPU, data-parallel:
    # one process per GPU, the gradients and stage-1 normalisers all-reduced over RCCL
    "c4": (8192, {"stage1": True, "mfma_dtype": "bf16x6", "start_it": 30000, "train_cfg": dict(C3_TRAIN)},
           "C4: Co3D/skateboard stage 1 on a synthetic 10-frame scene (MotionNetwork pose optimisation, scene-flow SDF "
           "loss, flow-RGB warp, SDF consistency with pose gradient), 8192 rays x 128 samples per GPU, fp32 (bf16x6), "
           "data-parallel (RCCL all-reduce of the gradients and the stage-1 normalisers)"),
    "c5": (4096, {"ren_cfg": dict(n_samples=64, n_importance=128, n_outside=0, up_sample_steps=4, perturb=1.0,
                                  n_max_network_queries=64000, importance_sampling_start=0, naive_render=False),
                  "graph": True, "mfma_dtype": "bf16x6"},
           "C5: synthetic scene, 4096 rays x 192 samples (coarse 64 + fine 4x32), fp32, HIP-graph-captured step"),
}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, rendezvous on 127.0.0.1) and
    return the exit status.  Runs before anything touches the GPU: the parent only waits, so no
    process that initialised HIP ever starts another program.  If one rank fails the others are
    stopped (by their exact pids) and its status is returned."""
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    if status != 0:  # every rank's exit status (a rank stopped by the parent shows its signal)
        print(f"bench.py: rank exit statuses {[p.returncode for p in procs]}", file=sys.stderr, flush=True)
    return status


def init_group(backend, rank, world, timeout_s, **kw):
    """init_process_group with a timeout on the rendezvous and on every collective (RCCL's watchdog
    tears the process down when one hangs), so a rank that never joins or a stuck all-reduce ends
    the run with a message and a non-zero status instead of at the driver's limit."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "3")  # a timed-out collective ends the process
    try:
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    except Exception as e:  # (the store raises its own timeout / connection types)
        print(f"bench.py rank {rank}: the {world}-rank process group did not form within {timeout_s:.0f} s: "
              f"{type(e).__name__}: {e}", file=sys.stderr, flush=True)
        sys.exit(3)


def dry_step(rank, world, grad_numel=800_000):
    """--dry: the launcher / process-group / timing plumbing with no HIP work (CPU tensors, gloo):
    a small CPU computation and the flat gradient all-reduce of the real step's size (~3.2 MB)."""
    g = torch.Generator().manual_seed(rank)
    a = torch.rand(256, 256, generator=g)
    flat = (a @ a).flatten().repeat(grad_numel // a.numel() + 1)[:grad_numel]
    if world > 1:
        dist.all_reduce(flat)
        flat /= world
    return flat.sum()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks) of this node; without WORLD_SIZE in the environment bench.py starts them "
                         "itself (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2")
    ap.add_argument("--rays", type=int, default=None, help="rays per GPU (default: the config's)")
    ap.add_argument("--graph", action="store_true", help="replay the step from a captured HIP graph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timer-steps", type=int, default=3, help="instrumented steps after the timed ones (roofline)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend (nccl = RCCL over xGMI; gloo only with --dry)")
    ap.add_argument("--dry", action="store_true",
                    help="launcher check on the CPU: ranks, process group, barriers and timing without HIP work")
    ap.add_argument("--pg-timeout", type=float, default=120.0,
                    help="seconds a rank waits for the process group to form or for a collective before it exits "
                         "non-zero (well inside the driver's limit)")
    ap.add_argument("--dry-absent-rank", type=int, default=-1, help=argparse.SUPPRESS)  # test hook (--dry only)
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} in the environment")
    if args.backend == "gloo" and not args.dry:
        sys.exit("bench.py: --backend gloo is for --dry runs only (the HIP path all-reduces over RCCL)")
    rays_cfg, kw, workload = CONFIGS[args.config]
    kw = dict(kw)
    graph = kw.pop("graph", False) or args.graph
    rays = args.rays or rays_cfg

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # COPENERF_FORCE_DIST=1 runs the RCCL path (process group + flat all-reduce) even at one rank
    distributed = world > 1 or os.environ.get("COPENERF_FORCE_DIST") == "1"
    if args.dry:
        return dry_main(args, world, rank, distributed)
    torch.cuda.set_device(local)
    if distributed:
        init_group("nccl", rank, world, args.pg_timeout, device_id=torch.device("cuda", local))
        joined = torch.ones(1, device=f"cuda:{local}")
        dist.all_reduce(joined)
        if int(joined.item()) != world:
            raise RuntimeError(f"{int(joined.item())} of {world} ranks joined the process group")

    from copenerf import ops
    from copenerf.train_step import GraphedTrainer, SyntheticTrainer
    infer = kw.pop("infer", False)
    mode = kw.get("mfma_dtype", "fp32")
    tr = SyntheticTrainer(f"cuda:{local}", rays=4096 if infer else rays, distributed=distributed and not infer,
                          capturable=graph, **kw)
    step = tr.step
    if infer:
        from copenerf.inference import render_image
        t_img = torch.zeros(1, device=f"cuda:{local}")

        def step():
            out = render_image(tr.renderer, tr.K, tr.I, tr.I, (tr.H, tr.W), t_img, chunk=65536)
            return out["rgb"].sum()
    if graph:  # the captured step includes the data-parallel all-reduce (RCCL) when distributed
        g = GraphedTrainer(tr, warmup=max(1, args.warmup))
        step = g.step

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], device=f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    if not torch.isfinite(loss).item():
        raise RuntimeError("non-finite loss in the timed steps")
    # the roofline pass: separate, instrumented (HIP events around every GEMM), eager
    timer = ops.KernelTimer()
    ops.set_kernel_timer(timer)
    n_inst = max(1, args.timer_steps)
    for _ in range(n_inst):
        tr.step() if not infer else step()
    torch.cuda.synchronize()
    ops.set_kernel_timer(None)

    rays_total = rays * world * args.steps
    S = 192 if args.config == "c5" else SAMPLES
    metric = "rays/sec (train step incl. backward) at 4096 rays × 128 samples"
    if args.config != "c2" or rays != RAYS:
        metric = f"rays/sec (train step incl. backward) at {rays} rays × {S} samples ({args.config})"
    if infer:
        metric = f"rays/sec (inference render, forward only) at 540x960 × {S} samples"
    result = {
        "metric": metric,
        "value": round(rays_total / elapsed, 1),
        "unit": "rays/s",
        "n_gpus": world,
        "ranks_joined": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16 MFMA operands, fp32 accumulate/activations" if mode == "bf16" else "fp32",
        "data": "synthetic (10 random 540x960 frames cycled one per step, 4x4 patches, " +
                ("learnable SE(3) poses" if kw.get("joint_pose") else
                 "identity camera, camera motion learned by the MotionNetwork (stage 1)" if kw.get("stage1") else
                 "fixed identity pose") +
                ", geometric-init SDF, seed 678)",
        "config": {"workload": workload, "gemm": MODE_TEXT[mode], "rays_per_gpu": rays, "samples_per_ray": S,
                   "global_rays": rays * world, "hip_graph": graph,
                   "parallelism": f"dp{world}" if world > 1 else "single"},
        "roofline": None,
        "cpu_baseline": None,
    }
    result.update(roofline_fields(timer, n_inst, rays_total / elapsed, mode, args.config))
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c2":
        result["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.destroy_process_group()


def dry_main(args, world, rank, distributed):
    """The --dry line: same launch, barriers and max-over-ranks timing as the HIP bench, CPU work."""
    if distributed:
        if rank == args.dry_absent_rank:  # (test hook) this rank never joins: the others must time out
            time.sleep(10 * args.pg_timeout)
            sys.exit(1)
        init_group(args.backend, rank, world, args.pg_timeout)
        joined = torch.ones(1)
        dist.all_reduce(joined)
        if int(joined.item()) != world:
            raise RuntimeError(f"{int(joined.item())} of {world} ranks joined the process group")
    for _ in range(args.warmup):
        dry_step(rank, world)
    if distributed:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dry_step(rank, world)
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    if rank == 0:
        print(json.dumps({"metric": "dry launcher check (no HIP work)", "value": round(args.steps * world / elapsed, 1),
                          "unit": "steps/s", "n_gpus": world, "ranks_joined": world, "steps": args.steps,
                          "warmup": args.warmup, "backend": args.backend if distributed else None,
                          "config": {"parallelism": f"dp{world}" if world > 1 else "single"}}), flush=True)
    if distributed:
        dist.destroy_process_group()


def roofline_fields(timer, steps, rays_per_s, mode, config="c2"):
    agg = timer.summary()
    # the dominant launch class over every cn_linear and cn_wgrad class (a launch class is one
    # kernel instance, named by the library: cn_linear_kernel_name / cn_wgrad_kernel_name; a
    # cn_wgrad / cn_wgrad_batch call is its split-M MFMA kernel plus the fixed-order slab reduction,
    # both inside the class's HIP events)
    dom_key = max(agg, key=lambda k: agg[k]["ms"])
    dom = agg[dom_key]
    avg_s = dom["ms"] / dom["launches"] * 1e-3
    flops, nbytes = dom["flops"] / dom["launches"], dom["bytes"] / dom["launches"]
    peak_tf = MODE_PEAK_TFLOPS[mode]
    t_flop, t_byte = flops / (peak_tf * 1e12), nbytes / (HBM_PEAK_GBS * 1e9)
    hbm = t_byte > t_flop  # the binding ceiling: the larger of the two times
    symbol = timer.symbols[dom_key]
    traffic, traffic_src = pmc_traffic(symbol, lib_stamp())
    kernels_ms = sum(a["ms"] for a in agg.values()) / steps
    # the kernel's own duration from the committed rocprofv3 stats of this config (the HIP events
    # bracket the library call: for a weight gradient also its slab reduction); the HIP-event
    # figure of this run beside it
    frac_ev = max(t_flop, t_byte) / avg_s
    stamp = lib_stamp()
    prof_ns, prof_src = rocprof_launch_ns(symbol, config, stamp)
    kern_s = prof_ns * 1e-9 if prof_ns else avg_s
    roof = {"bound": "hbm" if hbm else "mfma",
            "achieved": round(nbytes / kern_s / 1e9, 1) if hbm else round(flops / kern_s / 1e12, 2),
            "peak": HBM_PEAK_GBS if hbm else round(peak_tf, 1), "unit": "GB/s" if hbm else "TFLOP/s",
            "frac": round(max(t_flop, t_byte) / kern_s, 4),
            "frac_source": (f"{prof_src}: the kernel's rocprofv3 average duration" if prof_src else
                            "HIP events of this run (no committed rocprofv3 stats of this library build name "
                            "this kernel)"),
            "lib_stamp": stamp,
            "avg_launch_ms_rocprof": round(prof_ns * 1e-6, 4) if prof_ns else None,
            "frac_hip_events": round(frac_ev, 4),
            "traffic": traffic, "traffic_source": traffic_src,
            "kernel": symbol, "launch_class": "/".join(map(str, dom_key)),
            "timed_region": ("the cn_wgrad_batch call (a backward pass's 256x256 weight gradients in one launch): "
                             "this kernel + one cn::slab_reduce_kernel (every job's dW, db)"
                             if "WgradBatch" in symbol else
                             "the cn_wgrad call: this kernel + cn::slab_reduce_kernel (dW, db)") if dom_key[0] == "wgrad"
            else "this kernel", "launches_per_step": dom["launches"] / steps, "avg_launch_ms": round(avg_s * 1e3, 4),
            "algorithmic_gflop_per_launch": round(flops / 1e9, 3),
            "algorithmic_mb_per_launch": round(nbytes / 1e6, 1),
            "tflops": round(flops / avg_s / 1e12, 2), "gbs": round(nbytes / avg_s / 1e9, 1),
            "frac_mfma": round(t_flop / avg_s, 4), "frac_hbm": round(t_byte / avg_s, 4),
            "peak_basis": {"fp32": "fp32 MFMA dense", "bf16": "bf16 MFMA dense",
                           "bf16x6": "bf16 MFMA dense / 6 products"}[mode] + "; HBM3E 8 TB/s"}
    return {
        "roofline": roof,
        "effective_ref_tflops": round(rays_per_s * GFLOP_PER_RAY_REF / 1e3, 2),
        "gemm_ms_per_step": round(kernels_ms, 3),
        "gemm_tflops_avg": round(sum(a["flops"] for a in agg.values()) / sum(a["ms"] for a in agg.values()) / 1e9, 2),
        "roofline_by_class": {"/".join(map(str, k)): {"tflops": round(v["flops"] / v["ms"] / 1e9, 1),
                                                       "gbs": round(v["bytes"] / v["ms"] / 1e6, 1),
                                                       "launches_per_step": round(v["launches"] / steps, 2),
                                                       "algorithmic_mb_per_launch":
                                                           round(v["bytes"] / v["launches"] / 1e6, 1)}
                              for k, v in sorted(agg.items(), key=lambda kv: -kv[1]["ms"])},
        "kernel_breakdown_ms_per_step": {"/".join(map(str, k)): round(v["ms"] / steps, 3) for k, v in
                                         sorted(agg.items(), key=lambda kv: -kv[1]["ms"])},
        "kernel_symbols": {"/".join(map(str, k)): timer.symbols[k] for k in agg},
    }


if __name__ == "__main__":
    main()
