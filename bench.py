"""Benchmark: ResNet-18 / CIFAR-100 DDP training step on MI355X (BASELINE.json metric).

One step = the reference DDP loop body (src/ddp/trainer.py:149-167): zero_grad, autocast
forward + CrossEntropy, dist.barrier(), scaler.scale(loss).backward() (bucketed RCCL all-reduce
overlapped inside the native backward), scaler.step (fused Nesterov SGD), scaler.update(),
loss.item(). Per-GPU batch is fixed (256 images of 3x32x32, BASELINE config 2 at N=1), so the
multi-GPU runs are weak-scaled; synthetic inputs are resident in HBM before timing starts.

Launch: `python bench.py` (N=1), `python bench.py --gpus N` (bench.py starts the N rank
processes itself, as ddp/main.py:46-49's mp.spawn does) or `python -m torch.distributed.run
--nproc-per-node N ... bench.py --gpus N`. The world size must equal --gpus. Rank 0 prints one
JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import dtc_import  # noqa: E402

BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA, MI355X_MICROARCH.md "Peak BF16/FP16 MFMA"
FLOPS_PER_IMAGE = 3_329_273_856  # conv + FC, fwd + dgrad + wgrad at 32x32


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_envs(n: int, port: int, base=None) -> list:
    """The environment of each of `n` rank processes on this node (torchrun's variables, rendezvous
    on 127.0.0.1): what ddp/main.py:46-49's mp.spawn + init_process_group(tcp://127.0.0.1) set up."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def spawn_ranks(n: int, argv: list, script: str = None, poll_s: float = 0.2) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (one per GPU,
    as the reference's ddp/main.py:46-49 mp.spawn does) BEFORE anything in this process touches the
    GPU, pass argv through unchanged, and wait. Rank 0's stdout (the JSON line) is inherited. If a rank
    fails, the others are terminated by PID and the first failing exit status is returned."""
    import subprocess

    script = script or os.path.abspath(__file__)
    procs = [subprocess.Popen([sys.executable, script] + list(argv), env=e)
             for e in rank_envs(n, _free_port())]
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                for q in live:  # a rank died: the rest would wait in a collective forever
                    q.terminate()
        time.sleep(poll_s)
    return rc


def visible_gpus(env=None, kfd="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs this process could use, counted WITHOUT the HIP runtime (the launcher must not
    initialise the GPU before it starts the rank processes): the length of a *_VISIBLE_DEVICES list if
    one is set, else the KFD topology nodes with SIMDs (GPU agents; CPU nodes report simd_count 0).
    None when neither is available: the ranks then report a missing device themselves."""
    env = os.environ if env is None else env
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(k)
        if v is not None:
            return len([d for d in v.split(",") if d.strip() != ""])
    try:
        n = 0
        for node in os.listdir(kfd):
            with open(os.path.join(kfd, node, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if line.strip())
            if int(props.get("simd_count", "0")) > 0:
                n += 1
        return n
    except (OSError, ValueError):
        return None


def init_dist(gpus: int = 1):
    if "RANK" not in os.environ:  # one rank, no launcher: an in-process store (no TCP port to race for)
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0), store=dist.HashStore(), rank=0,
                                world_size=1)
        check_world(dist.get_world_size(), gpus)
        return 0, 1, 0
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    check_world(dist.get_world_size(), gpus)
    return dist.get_rank(), dist.get_world_size(), local


def check_world(world: int, gpus: int) -> None:
    """--gpus N must be the job's world size: a run that times fewer ranks than it claims is refused."""
    if world != gpus:
        raise SystemExit(f"bench.py: world size {world} != --gpus {gpus} (launch with --gpus {world}, or let "
                         f"bench.py start the ranks itself: `python bench.py --gpus {gpus}`)")


BN_IDEAL_BYTES_PER_IMAGE = 6.144e6  # non-GEMM HBM bytes per 32x32 image at ideal fusion


def profile_order_key(name: str):
    """Sort key of a committed profile file name, oldest first: round number, then the session tag in
    the order the tags were handed out (a..z, then aa..az, ...: shorter tags are older), e.g.
    r04u_... < r04ad_... < r05a_... (a plain lexicographic sort put r04u after r04ad: VERDICT r4 weak 6)."""
    import re

    m = re.match(r"r(\d+)_?([a-z0-9]*?)_", os.path.basename(name))
    if not m:
        return (-1, 0, "")
    return (int(m.group(1)), len(m.group(2)), m.group(2))


TRAFFIC_WORKLOAD = (256, 32)  # (per-GPU batch, image size) of tools/pmc_bench.sh's bench.py run


def committed_traffic(batch: int, size: int, path: str = None):
    """(HBM bytes per conv call, source) from a committed PMC summary (profiles/*conv_traffic.json, written
    by tools/pmc_traffic.py from rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py's default workload).
    PMC counters cannot be read live, so the value is the profile's and `source` names the file: `path` if
    given, else the newest by round and session (profile_order_key). None for another workload: the file
    measured B=256 at 32x32 only."""
    import glob

    if path is None:
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*conv_traffic.json")), key=profile_order_key)
        if not files:
            return None, None
        path = files[-1]
    src = os.path.relpath(path, ROOT)
    if (batch, size) != TRAFFIC_WORKLOAD:
        return None, f"{src} measured batch {TRAFFIC_WORKLOAD[0]} at {TRAFFIC_WORKLOAD[1]}x{TRAFFIC_WORKLOAD[1]}: not this workload"
    try:
        return round(json.load(open(path))["hbm_bytes_per_call"], 1), src
    except Exception as e:
        return None, f"{src}: unreadable ({e!r})"


def comm_fields(bucket_us, exposed_us, steps, buckets_mb):
    """The rank's communication timing (dtc_rn18_comm_timing_result) as the JSON fields VERDICT r4 item 6
    asks for: `comm_exposed_us` -- how long the compute stream waited on communication per step: the tail
    from the last backward kernel to the Reducer's join (the last bucket's collective), plus the wait for the
    weight-gradient stream (earlier buckets' collectives and the remaining weight gradients) before the stem
    weight gradient -- and `buckets_us`, per bucket (issue order) the collective's start / end offset from the
    backward's start and its duration (timing events on the stream it runs on)."""
    if not steps:
        return None, None
    opt = lambda v: round(v, 2) if v >= 0 else None  # -1: no timed step recorded a tail (replayed backwards)
    exposed = {"tail_us": opt(exposed_us[0]), "side_join_us": round(exposed_us[1], 2),
               "total_us": opt(exposed_us[2]), "backward_us": round(exposed_us[3], 2), "steps": int(steps),
               "note": "tail = last backward kernel -> the Reducer's join on the compute stream (the last bucket's "
                       "collective, nothing left to overlap); side_join = the compute stream's wait for the "
                       "weight-gradient stream (its queued weight gradients + the earlier buckets' collectives) "
                       "before the stem weight gradient"}
    buckets = [{"bucket": i, "mb": (buckets_mb[i] if i < len(buckets_mb) else None),
                "start_us": round(bucket_us[3 * i], 2), "end_us": round(bucket_us[3 * i + 1], 2),
                "duration_us": round(bucket_us[3 * i + 2], 2)} for i in range(len(buckets_mb))]
    return exposed, buckets


def host_cores() -> dict:
    """The host's CPU inventory (state physical cores beside the thread count): logical
    CPUs, the CPUs this process may run on (affinity), and physical cores / sockets from
    /proc/cpuinfo ("physical id", "core id" pairs), counted over the whole machine and over the
    affinity set."""
    out = {"logical_cpus": os.cpu_count()}
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        aff = list(range(os.cpu_count() or 1))
    out["affinity_cpus"] = len(aff)
    try:
        cores, cores_aff, cpu, phys = set(), set(), None, None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "processor":
                cpu, phys = int(v), None
            elif k == "physical id":
                phys = int(v)
            elif k == "core id" and cpu is not None:
                key = (phys, int(v))
                cores.add(key)
                if cpu in aff:
                    cores_aff.add(key)
        if cores:
            out["physical_cores"] = len(cores)
            out["sockets"] = len({p for p, _ in cores})
            out["physical_cores_in_affinity"] = len(cores_aff)
    except OSError:
        pass
    out["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    return out


def cpu_baseline(seconds: float, steps: int = 50):
    """BASELINE config 1 on the host cores: the reference's single-device fp32 step
    (single/trainer.py:131-147) in stock torch CPU at batch 128 (oracle/torch_ref.py, pinned to the
    reference-produced fixture by tests/test_oracle_golden.py), 3 warm-up steps, then the median of
    up to `steps` steps bounded by `seconds` of CPU work. Threads = torch's intra-op pool
    (OMP_NUM_THREADS on the box: the cores this job may use)."""
    from oracle.torch_ref import time_cpu_step

    torch.manual_seed(42)
    dtc = dtc_import.load()
    m = dtc.ResNet18()  # host-side construction only (identical init to the reference)
    r = time_cpu_step(m.state_dict(), batch=128, warmup=3, steps=steps, max_seconds=seconds)
    return {"value": round(r["img_per_s"], 3), "unit": "images/sec", "cores": r["threads"], "kind": "port",
            "impl": "torch-cpu", "batch": 128, "dtype": "fp32", "host": host_cores(),
            "sample": f"config 1: median of {r['steps']} steps (after 3 warm-ups) of the single-device fp32 "
                      f"train step (zero_grad, forward, CrossEntropy, backward, SGD nesterov) at batch 128, "
                      f"32x32, stock torch {torch.__version__} CPU on {r['threads']} threads (the job's CPU "
                      f"share; host inventory in `host`); "
                      f"median step {r['median_s'] * 1e3:.1f} ms, {r['seconds']:.1f} s sampled"}


def bench_dp(args):
    """BASELINE config 4: DataParallel (src/dp/trainer.py:27) -- ONE process driving every GPU in
    --dp-devices (default: the first --gpus devices), global batch --batch split across them, the
    reference DP step (zero_grad, autocast forward, CE, scaler.scale(loss).backward(), step,
    update, loss.item()) with replicate / scatter / gather / reduce-add each step. Prints one
    JSON line; `value` is global images/s (strong scaling: total batch fixed)."""
    dev_ids = [int(d) for d in args.dp_devices.split(",")] if args.dp_devices else list(range(args.gpus))
    dev = torch.device("cuda", dev_ids[0])
    torch.cuda.set_device(dev)
    dtc = dtc_import.load()
    for kv in args.opt:
        name, val = kv.split("=")
        dtc._native.call("dtc_set_option", name.encode(), int(val))
    torch.manual_seed(42)
    model = dtc.DataParallel(dtc.ResNet18().to(dev), device_ids=dev_ids)
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.1, weight_decay=1e-4, momentum=0.9, nesterov=True)
    scaler = dtc.GradScaler()
    B, S = args.batch, args.size
    templates = dtc.data.class_templates(100, S, S)
    pool = [dtc.data.synthetic_batch(i, B, S, S, 100, dev, templates) for i in range(4)]
    losses = []

    def step(i):
        img, label = pool[i % len(pool)]
        opt.zero_grad()
        with dtc.autocast():
            loss = crit(model(img), label)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        losses.append(loss.item())

    for i in range(args.warmup):
        step(i)
    for d in set(dev_ids):
        torch.cuda.synchronize(d)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    for d in set(dev_ids):
        torch.cuda.synchronize(d)
    elapsed = time.perf_counter() - t0
    shared = len(set(dev_ids)) < len(dev_ids)
    print(json.dumps({
        "metric": f"images/sec ResNet-18 CIFAR-100 DataParallel (global batch {B}, one process)",
        "value": round(B * args.steps / elapsed, 2), "unit": "images/sec", "n_gpus": len(set(dev_ids)),
        "replicas": len(dev_ids), "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic, resident in HBM",
        "config": {"workload": f"ResNet-18 DataParallel step, global batch {B}, {S}x{S}", "model": "ResNet18",
                   "global_batch": B, "seq_len": None, "parallelism": f"dp-single-process x{len(dev_ids)}",
                   "device_ids": dev_ids,
                   "transport": "replicas share one device: on-device copies + HIP reduce-add (dtc_dp_*)" if shared
                   else "grouped RCCL broadcast / reduce over distinct devices (dtc_dp_*, ncclCommInitAll)"},
        "note": (f"device_ids {dev_ids}: {len(dev_ids)} replicas on ONE GPU -- the single-GPU form of the "
                 "DataParallel path, NOT BASELINE config 4 (8 GPUs)") if shared else None,
        "final_loss": round(losses[-1], 4)}), flush=True)


HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); measured copy ~6.3 TB/s


def hbm_probe(dtc, dev, B, S, nparam, reps=20):
    """Achieved HBM GB/s of the two HBM-bound kernel classes the north star names, timed with
    device events on the stream they are launched on (torch's current stream), after the timed
    regions: (1) the stand-alone dtc_bn_bwd_reduce (bf16-output mask, dz stored: 8 B/element) at the
    largest BN shape of the step (B*S*S pixels x 64 channels) -- an isolated bandwidth reference; the
    executor's own BN kernels (mask-bit path) are timed in the step itself (`bn_in_step`); (2) the
    fused SGD-Nesterov + bf16-shadow kernel over a flat buffer of the model's size (reads p, g, m;
    writes p, m, bf16 p: 22 B/parameter), which the in-step timing does not cover. Scratch tensors."""
    ops = dtc.ops
    M, Cc = B * S * S, 64
    g = torch.Generator(device=dev).manual_seed(7)
    dy = torch.randn(M, Cc, device=dev, generator=g).bfloat16()
    y = torch.randn(M, Cc, device=dev, generator=g).bfloat16()
    x = torch.randn(M, Cc, device=dev, generator=g).bfloat16()
    mean = torch.zeros(Cc, device=dev)
    invstd = torch.ones(Cc, device=dev)
    p = torch.randn(nparam, device=dev, generator=g)
    gr = torch.randn(nparam, device=dev, generator=g) * 1e-3
    mom = torch.zeros(nparam, device=dev)
    pb = torch.empty(nparam, dtype=torch.bfloat16, device=dev)

    def timeit(fn):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3 / reps

    acc = ops.new_stats(Cc, dev)
    dz = torch.empty_like(dy)
    P, sp, call = dtc._native.ptr, dtc._native.stream_ptr, dtc._native.call
    # the C-ABI directly with preallocated outputs (the slots accumulate across launches: only timing here)
    t_bn = timeit(lambda: call("dtc_bn_bwd_reduce", P(dy), P(y), P(x), P(mean), P(invstd), P(acc), None, None, None,
                               None, P(dz), M, Cc, sp()))
    t_sgd = timeit(lambda: ops.sgd_nesterov_flat(p, gr, mom, pb, 1e-3, 1e-4, 0.9))
    out = {}
    for name, t, nbytes, unit in (("bn_bwd_reduce", t_bn, 8 * M * Cc, f"{M}x{Cc} bf16, 8 B/element"),
                                  ("sgd_nesterov", t_sgd, 22 * nparam, f"{nparam} params, 22 B/param")):
        gbps = nbytes / t / 1e9
        out[name] = {"us": round(t * 1e6, 2), "bytes": nbytes, "achieved_GBps": round(gbps, 1),
                     "peak_GBps": HBM_PEAK_GBPS, "frac": round(gbps / HBM_PEAK_GBPS, 4), "work": unit}
    out["timing"] = "device events on torch's current stream (the launch stream), mean of %d launches" % reps
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="BASELINE config 3: global batch split over the ranks, per-rank int(G/W) "
                         "(ddp/trainer.py:34; strong scaling)")
    ap.add_argument("--sim-world", type=int, default=1,
                    help="N=1 only: run ONE rank of a W-rank job -- per-rank batch int(G/W) with --global-batch, "
                         "gradients pre-scaled 1/W and the bucketed all-reduce backward forced on (a one-rank RCCL "
                         "communicator): the per-rank shape and code path of config 3 measured on one GPU")
    ap.add_argument("--sim-comm", choices=("rccl", "loopback"), default="rccl",
                    help="--sim-world's communicator: the one-rank RCCL communicator (RCCL special-cases one rank: "
                         "no kernel, host-side copies) or the loopback communicator (an identity scale kernel per "
                         "bucket on the collective's side stream: the executor's own overlap cost, no RCCL)")
    ap.add_argument("--no-config3", action="store_true",
                    help="N>1: skip the extra config-3 region (global batch 256 over the ranks)")
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--no-barrier", action="store_true", help="drop the reference's per-step dist.barrier()")
    ap.add_argument("--torch-barrier", action="store_true", help="per-step barrier via torch.distributed (A/B)")
    ap.add_argument("--no-item", action="store_true", help="drop the per-step loss.item() host sync")
    ap.add_argument("--cpu-seconds", type=float, default=30.0, help="bound on the timed CPU-baseline steps")
    ap.add_argument("--cpu-steps", type=int, default=50, help="CPU baseline: median over this many steps")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-live-roofline", action="store_true", help="skip the per-conv timing in the timed region")
    ap.add_argument("--mode", choices=("ddp", "dp"), default="ddp",
                    help="dp: BASELINE config 4, single-process DataParallel (global --batch over --gpus devices)")
    ap.add_argument("--dp-devices", default="", help="dp mode: comma-separated replica devices (may repeat)")
    ap.add_argument("--no-allreduce-probe", action="store_true", help="skip the N>1 all-reduce busBW probe")
    ap.add_argument("--no-comm-timing", action="store_true",
                    help="skip the per-bucket / exposed-communication timing region (N>1 or --sim-world)")
    ap.add_argument("--allreduce-probe", action="store_true", help="run the busBW probe at N=1 too (plumbing check)")
    ap.add_argument("--no-hbm-probe", action="store_true", help="skip the BN / SGD HBM-roofline probe")
    ap.add_argument("--sync-bn", action="store_true",
                    help="SyncBatchNorm (off in the reference); at N=1 a one-rank communicator forces the sync path")
    ap.add_argument("--opt", action="append", default=[], help="native option NAME=VALUE (A/B runs)")
    ap.add_argument("--traffic-file", default=None,
                    help="PMC conv-traffic summary for roofline.traffic (default: the newest profiles/*conv_traffic.json)")
    ap.add_argument("--stream-prio", type=int, default=0,
                    help="run the step on a torch stream of this priority (-1 = high; 0 = torch's default stream)")
    args = ap.parse_args()
    if args.mode == "dp":
        return bench_dp(args)
    if args.gpus > 1 and "RANK" not in os.environ:
        # no launcher: start the ranks here, before anything in this process touches HIP
        have = visible_gpus()
        if have is not None and have < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) visible")
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    rank, world, local = init_dist(args.gpus)
    dev = torch.device("cuda", local)
    dtc = dtc_import.load()
    for kv in args.opt:
        name, val = kv.split("=")
        dtc._native.call("dtc_set_option", name.encode(), int(val))

    torch.manual_seed(42)
    model = dtc.ResNet18().to(dev)
    if args.sync_bn:
        model = dtc.SyncBatchNorm.convert_sync_batchnorm(model)
    model = dtc.DDP(model, device_ids=[local], find_unused_parameters=True, bucket_cap_mb=args.bucket_mb)
    if args.sync_bn and world == 1:  # torch keeps local statistics at W=1; force the path to time it
        model.sync_comm = dtc.parallel.Comm(0, 1, dtc.parallel.Comm.unique_id(), local)
        model.module.set_sync_bn(model.sync_comm)
    sim = max(1, args.sim_world) if world == 1 else 1
    if sim > 1:  # one rank of a sim-rank job: 1/W pre-scale, bucketed all-reduce backward on the side stream
        model.module._comm = (dtc.parallel.Comm.loopback(local, factor=1.0, world=sim) if args.sim_comm == "loopback"
                              else model.comm)
        model.module._grad_scale = 1.0 / sim
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.1, weight_decay=1e-4, momentum=0.9, nesterov=True)
    scaler = dtc.GradScaler()

    ranks_of_job = world * sim
    B = int(args.global_batch / ranks_of_job) if args.global_batch else args.batch  # ddp/trainer.py:34
    S = args.size
    templates = dtc.data.class_templates(100, S, S)

    def make_pool(b):
        pool = []
        for i in range(4):
            x, y = dtc.data.synthetic_batch(1000 * rank + i, b, S, S, 100, dev, templates)
            pool.append((x.contiguous(), y.contiguous()))
        return pool

    pools = {B: make_pool(B)}
    losses = []
    if args.stream_prio:  # A/B: the caller's stream (the executor's main chain) at another hardware priority
        torch.cuda.synchronize()
        torch.cuda.set_stream(torch.cuda.Stream(dev, priority=args.stream_prio))

    def step(i, b=B, host_sync=True):
        img, label = pools[b][i % len(pools[b])]
        opt.zero_grad()
        with dtc.autocast():
            logit = model(img)
            loss = crit(logit, label)
        if host_sync and not args.no_barrier:
            if args.torch_barrier:
                dist.barrier()
            else:
                dtc.barrier()  # the reference's dist.barrier() (trainer.py:156) on the native communicator
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        if host_sync and not args.no_item:
            losses.append(loss.item())

    def timed(k, first, b=B, host_sync=True):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            step(first + i, b, host_sync)
        torch.cuda.synchronize()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)  # the slowest rank defines the step time
        return float(el.item())

    for i in range(args.warmup):
        step(i)
    # Region 1 (the reported value): K plain steps.
    elapsed = timed(args.steps, args.warmup)
    # Region 2 (roofline): the same K steps, serialized and eager (options bwd_streams=0, graphs=0: every
    # kernel has the chip to itself and is launched on the compute stream), with every timed launcher call
    # bracketed by two HIP timing events on that stream (dtc_rn18_profile_events: its launch duration as
    # the rocprofv3 kernel trace of the same command -- `--opt bwd_streams=0 --opt graphs=0` -- sees it).
    # The kernels' own s_memrealtime stamps (first workgroup start .. last workgroup end, folded on the
    # device) are kept beside them as `stamp_*`. Two untimed steps follow the arming; totals re-zeroed.
    import ctypes as C
    ms4, fl4, cnt4 = (C.c_double * 4)(), (C.c_double * 4)(), (C.c_int * 4)()  # events
    sms4, sfl4, scnt4 = (C.c_double * 4)(), (C.c_double * 4)(), (C.c_int * 4)()  # stamps
    prof_elapsed = None
    ev_dropped = C.c_int64(0)  # timed calls the event pool could not bracket: the totals then undercount
    if not args.no_live_roofline:
        exe = model.module.executor(B, S, S, "bf16")
        saved = {k: int(dtc._native.lib.dtc_get_option(k)) for k in (b"bwd_streams", b"graphs")}
        dtc._native.call("dtc_set_option", b"bwd_streams", 0)
        dtc._native.call("dtc_set_option", b"graphs", 0)
        dtc._native.call("dtc_rn18_profile_begin", exe.handle, 1)
        dtc._native.call("dtc_rn18_profile_events", exe.handle, 256 * 2)
        for i in range(2):
            step(args.warmup + args.steps + i)
        torch.cuda.synchronize()
        dtc._native.call("dtc_rn18_profile_begin", exe.handle, 1)
        dtc._native.call("dtc_rn18_profile_events", exe.handle, 256 * (args.steps + 1))
        # (no per-step barrier / loss.item() host sync in this region: the host stays ahead of the GPU,
        # so an event pair times its launch, not a launch plus the host catching up after a drain)
        prof_elapsed = timed(args.steps, args.warmup + args.steps + 2, host_sync=False)
        dtc._native.call("dtc_rn18_profile_events_result", exe.handle, 4, ms4, fl4, cnt4)
        dtc._native.call("dtc_rn18_profile_events_dropped", exe.handle, C.byref(ev_dropped))
        dtc._native.call("dtc_rn18_profile_end_ex", exe.handle, 4, sms4, sfl4, scnt4)
        for k, v in saved.items():
            dtc._native.call("dtc_set_option", k, v)
    ms, fl, cnt = list(ms4)[:3], list(fl4)[:3], list(cnt4)[:3]  # the conv passes (kinds 0-2)

    # Communication timing (N > 1 or --sim-world): the same K steps again with timing events around every
    # bucket collective and at the backward's joins (dtc_rn18_comm_timing), after the timed regions so the
    # events never perturb `value`; rank 0 reports its own rank's figures
    comm_exposed, buckets_us = None, None
    if model.module._comm is not None and not args.no_comm_timing:
        exe = model.module.executor(B, S, S, "bf16")
        nb = len(model.buckets)
        dtc._native.call("dtc_rn18_comm_timing", exe.handle, args.steps)
        for i in range(args.steps):
            step(args.warmup + i)
        torch.cuda.synchronize()
        bus, exu, nst = (C.c_double * (3 * max(1, nb)))(), (C.c_double * 5)(), C.c_int(0)
        dtc._native.call("dtc_rn18_comm_timing_result", exe.handle, nb, bus, exu, C.byref(nst))
        comm_exposed, buckets_us = comm_fields(list(bus), list(exu), nst.value,
                                               [round(n * 4 / 2**20, 2) for _, n in model.buckets])

    # BASELINE config 3 beside the weak-scaled value at N > 1: the reference's own DDP job, global
    # batch 256 over the ranks (per-rank int(256/W), ddp/trainer.py:34, run_ddp.sh:4) -- strong scaling
    config3 = None
    if world > 1 and not args.global_batch and not args.no_config3:
        b3 = int(256 / world)
        pools[b3] = make_pool(b3)
        for i in range(5):
            step(i, b3)
        e3 = timed(args.steps, 5, b3)
        config3 = {"workload": f"BASELINE config 3: global batch 256 over {world} ranks ({b3}/GPU), 32x32 bf16",
                   "global_batch": b3 * world, "per_gpu_batch": b3, "scaling": "strong",
                   "value": round(b3 * world * args.steps / e3, 2), "unit": "images/sec",
                   "ms_per_step": round(e3 / args.steps * 1e3, 4), "steps": args.steps, "warmup": 5}

    # C4 all-reduce bus bandwidth on the Reducer's own RCCL communicator: the full gradient
    # (11,220,132 fp32) and the bucket-size sweep of BASELINE config 5 (N > 1 only: one rank has
    # no exchange). Runs after both timed regions, so it never overlaps the measured steps.
    allreduce = None
    if (world > 1 or args.allreduce_probe) and not args.no_allreduce_probe:
        par = dtc.parallel
        try:
            grad_bytes = int(model.module.flat.grads.numel()) * 4
            allreduce = {"grad": par.allreduce_probe(model.comm.allreduce_sum_, grad_bytes, dev, world),
                         "sweep": [par.allreduce_probe(model.comm.allreduce_sum_, int(mb * 2**20), dev, world)
                                   for mb in (1, 2, 5, 10, 25, 50, 100)],
                         "transport": "native RCCL communicator (dtc_comm_allreduce_sum), fp32 SUM, device events",
                         "peak_model": "(W-1) x 153 GB/s xGMI links per GPU (fully connected 8-GPU node)"}
        except Exception as e:  # report, never hide; the throughput line stands on its own
            allreduce = {"error": repr(e)}

    hbm = None
    if rank == 0 and not args.no_hbm_probe:
        try:
            hbm = hbm_probe(dtc, dev, B, S, int(model.module.flat.params.numel()))
        except Exception as e:  # report, never hide
            hbm = {"error": repr(e)}

    if rank == 0:
        conv_ms = sum(ms)
        conv_flops = sum(fl)
        traffic, traffic_src = committed_traffic(B, S, args.traffic_file)
        n_launch = sum(cnt)
        # refuse a fraction whose time total misses launches (event pool used up) -- it would be overstated
        achieved = conv_flops / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 and ev_dropped.value == 0 else None
        value = B * world * args.steps / elapsed
        if args.global_batch:
            metric = (f"images/sec/node ResNet-18 CIFAR-100 DDP (global batch {args.global_batch} over "
                      f"{ranks_of_job} ranks, {B} images/GPU" + (")" if S == 32 else f", {S}x{S})"))
        else:
            metric = (f"images/sec/node ResNet-18 CIFAR-100 DDP (weak-scaled, {B} images/GPU"
                      + (")" if S == 32 else f", {S}x{S})"))
        workload = (f"ResNet-18 CIFAR-100 train step, batch {B}/GPU, {S}x{S}, bf16 MFMA, SGD-Nesterov + GradScaler, "
                    f"DDP bucket {args.bucket_mb} MB")
        if sim > 1:
            workload += (f"; ONE rank of a {sim}-rank job on 1 GPU (per-rank shape of BASELINE config 3, 1/{sim} "
                         f"pre-scale, bucketed all-reduce backward on a {'loopback' if args.sim_comm == 'loopback' else 'one-rank RCCL'} communicator): value is "
                         f"this rank's images/s, the node figure needs {sim} GPUs")
        out = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.global_batch else "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (0.5*class_template + N(0,1), 100 classes), resident in HBM",
            "config": {"workload": workload,
                       "model": "ResNet18 (CIFAR, src/ddp/net.py)", "global_batch": B * ranks_of_job, "seq_len": None,
                       "parallelism": f"dp{world}", "per_gpu_batch": B, "image_size": S,
                       "sim_world": sim,
                       "step_barrier": not args.no_barrier, "loss_item": not args.no_item,
                       "sync_bn": bool(args.sync_bn),
                       "buckets_mb": [round(n * 4 / 2**20, 2) for _, n in model.buckets]},
            "roofline": {
                "bound": "mfma",
                "achieved": round(achieved, 2) if achieved else None,
                "peak": BF16_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / BF16_PEAK_TFLOPS, 4) if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": "every conv launch of the step (stem, halo / c64 / implicit-GEMM fwd, dgrad, wgrad incl. "
                          "split-K and wgrad reductions); per-call duration = HIP timing events recorded on the "
                          "launch (compute) stream before and after the call, in a second timed region of the same "
                          "K steps run serialized and eager (bwd_streams=0, graphs=0: each launch has the chip to "
                          "itself) without the per-step host syncs (the host stays ahead; region_ms_per_step) -- reproduce with tools/prof_summary.py on a rocprofv3 "
                          "kernel trace of `bench.py --opt bwd_streams=0 --opt graphs=0`; value from the first "
                          "region (weight gradients overlapped on a side stream, the default launch mode)",
                "stamp_conv_ms_per_step": round(sum(list(sms4)[:3]) / args.steps, 4),
                "stamp_frac": (round(sum(list(sfl4)[:3]) / (sum(list(sms4)[:3]) * 1e-3) / 1e12 / BF16_PEAK_TFLOPS, 4)
                               if sum(list(sms4)[:3]) > 0 else None),
                "stamp_note": "kernel self-stamps (first workgroup start .. last workgroup end, s_memrealtime) of the "
                              "same calls: excludes each dispatch's ramp before its first workgroup",
                "traffic_unit": "HBM bytes per conv call (PMC, profiles/*conv_traffic.json)",
                "conv_ms_per_step": round(conv_ms / args.steps, 4),
                "region_ms_per_step": round(prof_elapsed / args.steps * 1e3, 4) if prof_elapsed else None,
                "conv_ms_by_pass": [round(v / args.steps, 4) for v in ms],
                "conv_calls_per_step": n_launch // max(1, args.steps),
                "unbracketed_calls": int(ev_dropped.value),
                "algorithmic_gflop_per_step": round(conv_flops / args.steps / 1e9, 3),
            },
            "hbm_roofline": hbm,
            # the whole in-step BN family (kind 3: forward finalize+apply, backward reduce, backward
            # finalize+apply of all 20 BNs), measured live in region 2 like the convs: algorithmic bytes
            # (each tensor read / written once) / summed kernel durations
            "bn_in_step": ({"ms_per_step": round(ms4[3] / args.steps, 4),
                            "stamp_ms_per_step": round(sms4[3] / args.steps, 4),
                            "timing": "HIP events around each BN launch, serialized eager region (as roofline)",
                            "bytes_per_step": round(fl4[3] / args.steps),
                            "calls_per_step": cnt4[3] // max(1, args.steps),
                            "achieved_GBps": round(fl4[3] / (ms4[3] * 1e-3) / 1e9, 1) if ms4[3] > 0 else None,
                            "peak_GBps": HBM_PEAK_GBPS,
                            "frac": round(fl4[3] / (ms4[3] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if ms4[3] > 0 else None,
                            # SURVEY §8(d)'s ideal non-GEMM bytes (every BN / ReLU / residual tensor touched once
                            # under ideal fusion: 6.144 MB per 32x32 image) over the same measured time -- the
                            # fraction a perfectly fused design would be charged with
                            "ideal_bytes_per_step": round(BN_IDEAL_BYTES_PER_IMAGE * (S * S / 1024) * B),
                            "frac_vs_ideal_bytes": (round(BN_IDEAL_BYTES_PER_IMAGE * (S * S / 1024) * B
                                                          / (ms4[3] / args.steps * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
                                                    if ms4[3] > 0 else None)}
                           if not args.no_live_roofline else None),
            "step_flop_fraction_of_peak": round(FLOPS_PER_IMAGE * (S * S / 1024) * B / (elapsed / args.steps) / 1e12
                                                / BF16_PEAK_TFLOPS, 4),
            "final_loss": round(losses[-1], 4) if losses else None,
        }
        if comm_exposed is not None:
            out["comm_exposed_us"] = comm_exposed
            out["buckets_us"] = buckets_us
        if allreduce is not None:
            out["allreduce"] = allreduce
        if config3 is not None:
            out["config3"] = config3
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.cpu_steps)
            except Exception as e:  # report, never hide
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
