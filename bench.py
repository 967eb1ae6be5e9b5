"""Benchmark: unet_resnet50 binary segmentation training, 512x512, batch 16 per GPU, bf16 (HIP path).

    python bench.py --gpus N --steps K --warmup W
    (N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

A step = zero_grad + forward + Lovasz-hinge loss + backward (+ RCCL gradient all-reduce when N>1) +
fused Adam on one synthetic batch already resident in HBM.  After one eager step and one recording
step (--plan 1, default) the steps are replays of the recorded launch sequence (unetseg_hip/plan.py):
every kernel of the step runs every time, on the same streams; only the Python that chose them is not
re-run (tests/test_gpu_plan.py: bit-identical to eager steps).  Adam and the re-pack of the conv weights
run per gradient bucket on the weight-gradient stream while backward continues (--overlap-adam 1,
FusedAdam(overlap=True)); every parameter is updated inside each timed step.  Rank 0 prints ONE JSON line.
`roofline` covers the dominant kernel (igemm_tn: conv fwd + dgrad), measured with HIP events around
each of its launches in one probe step right after the timed region.  `cpu_baseline` times the CPU
oracle (oracle/ref_cpu.py, fp32, the reference's op sequence) on the host on a bounded sample.
`configs` times BASELINE.json's other GPU configurations the same way in the same process (C4
attention_unet B=8 at N=1, C5 multitask_unet B=8 BCE + CE at every N); `card` records the GPU's
clocks / power in the middle of the timed region and its own bf16 GEMM and HBM copy rates, so a slow
box can be told from a code change; every configuration also records its card state during its own
timed steps and `host_enqueue_ms` (the host's cost of enqueueing one step with the GPU parked, after
the timed region, N=1), so a host-bound rate can be told from a slow GPU.  `median_gpu_ms_per_step` is the median of per-step HIP-event
times over the K timed steps.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec training unet_resnet50 512×512 bf16 at 1/2/4/8 GPUs; mIoU parity"
GFLOP_PER_IMG = {"unet_resnet50": 547.46, "multitask_unet": 547.36, "attention_unet": 1374.35, "unet_plain": 83.48}
PEAK_BF16_TFLOPS = 2516.6  # gfx950 dense bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense)
HBM_PRACTICAL = 6.3e12  # B/s: what a streaming kernel reaches on this card (tools/hbm_bw.py), the floors' HBM rate


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="unet_resnet50")
    ap.add_argument("--batch", type=int, default=16, help="per-GPU batch")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--loss", default="lovasz_hinge")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 (N=1)")
    ap.add_argument("--cpu-batch", type=int, default=4, help="images in the bounded CPU sample")
    ap.add_argument("--probe", type=int, default=1)
    ap.add_argument("--graph", type=int, default=0, help="replay the whole step (fwd+loss+bwd+Adam) as a HIP graph")
    ap.add_argument("--stream", type=int, default=1, help="run the steps on a created (non-default) HIP stream")
    ap.add_argument("--priority", type=int, default=0, help="priority of that stream (lower = higher priority)")
    ap.add_argument("--overlap-adam", type=int, default=1,
                    help="Adam + weight re-pack per gradient bucket on the weight-gradient stream during backward")
    ap.add_argument("--bucket-mb", type=float, default=8.0, help="gradient bucket size (MB)")
    ap.add_argument("--extra-configs", type=int, default=1,
                    help="also time C4 (attention_unet B=8, N=1 only) and C5 (multitask_unet B=8) after the headline")
    ap.add_argument("--card-probe", type=int, default=1, help="bf16 GEMM + HBM copy rate of this card (rank 0)")
    ap.add_argument("--host-probe", type=int, default=1,
                    help="host enqueue cost per step (parks the GPU on a spin kernel; 0 under a profiler)")
    ap.add_argument("--plan", type=int, default=1,
                    help="replay a recorded step plan (unetseg_hip/plan.py: the eager step's launches re-issued "
                         "from the host, every kernel every step) after one eager and one recording step")
    ap.add_argument("--ddp-bf16", type=int, default=0,
                    help="N>1: all-reduce bf16 copies of the gradient buckets (half the bytes; opt-in)")
    return ap.parse_args()


def _cpu_share():
    """(threads to use, host CPU model, CPUs visible, CPU share) -- os.cpu_count() is the whole
    machine on the GPU box; the process's affinity mask and cgroup quota give its share."""
    visible = os.cpu_count() or 1
    try:
        share = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        share = visible
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            share = min(share, max(1, int(-(-int(q) // int(per)))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return share, model, visible


def cpu_baseline(model_name, size, batch):
    """The oracle's train step (fwd + loss + bwd + Adam) on this host's cores, bounded sample, in the
    reference's CPU precision for the task: binary loops run under bf16 autocast
    on CPU (train.py:170 always builds a GradScaler object, utils/train_and_eval.py:218), the
    multitask loop in fp32 (train.py:243).  fp32 is timed for the binary models too."""
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    from utils.synthetic import make_batch

    threads, cpu_model, visible = _cpu_share()
    torch.set_num_threads(threads)
    multitask = model_name == "multitask_unet"
    kw = dict(num_classes=1) if multitask else dict(num_classes=2)
    params, buffers = ref_cpu.split_state(make_torch_state(ref_cpu.model_spec(model_name, **kw)))
    m1 = {k: torch.zeros_like(v) for k, v in params.items()}
    m2 = {k: torch.zeros_like(v) for k, v in params.items()}
    x, y, c = make_batch(batch, size, seed=99, with_cls=True)
    mask = (torch.rand(batch, 512, generator=torch.Generator().manual_seed(5)) >= 0.5).float()

    def timed(autocast):
        times = []
        for i in range(3):  # 1 warmup + 2 timed
            t0 = time.perf_counter()
            if multitask:
                _, _, grads = ref_cpu.train_step_multitask(params, buffers, x, y, c, mask, 1.0, "bce")
            else:
                _, _, grads = ref_cpu.train_step(model_name, params, buffers, x, y, "lovasz_hinge",
                                                 autocast_bf16=autocast)
            ref_cpu.adam_step(params, grads, m1, m2, i + 1, 1e-4)
            times.append(time.perf_counter() - t0)
        return min(times[1:])

    t_main = timed(not multitask)
    out = {"value": round(batch / t_main, 4), "unit": "images/s", "cores": threads, "kind": "port",
           "precision": "fp32" if multitask else "bf16 autocast (reference CPU default)",
           "host_cpu": cpu_model, "host_cpus_visible": visible}
    if not multitask:
        t32 = timed(False)
        out["fp32_value"] = round(batch / t32, 4)
    out["sample"] = (f"oracle {model_name} {size}x{size} batch {batch}, 1 warmup + 2 timed train steps "
                     f"(fwd+{'bce+ce' if multitask else 'lovasz'}+bwd+Adam) per precision, best step "
                     f"{t_main:.2f} s, {threads} threads (this process's CPU share of {visible}), "
                     f"torch {torch.__version__} CPU; a bounded sample: the GPU line runs the same model "
                     f"and size at its own batch, images/s per image either way")
    return out


def pmc_traffic(workload, kind):
    """HBM bytes per launch of `kind` from the committed PMC summary (tools/pmc_traffic.py), if one was
    measured for this exact workload; bench.py cannot profile itself, so the counters come from two
    separate rocprofv3 --pmc passes of this same command (profiles/README.md)."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload and kind in d.get("groups", {}):
            best = (round(d["groups"][kind]["traffic_bytes_per_launch"]), os.path.relpath(f, REPO))
    return best


def pmc_mfma(workload, kind):
    """MFMA busy fraction of `kind` from the committed PMC summary (tools/pmc_mfma.py) for this exact
    workload: SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) over the group's kernels."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_mfma.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        g = d.get("groups", {}).get(kind)
        if d.get("workload") == workload and g and g.get("mfma_busy") is not None:
            best = (round(g["mfma_busy"], 4), os.path.relpath(f, REPO))
    return best


def _pci_dir(dev):
    """sysfs directory of this process's GPU (matched by PCI bus id), or None"""
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = "%04x:%02x:%02x.0" % (getattr(p, "pci_domain_id", 0), p.pci_bus_id, p.pci_device_id)
        d = os.path.join("/sys/bus/pci/devices", bdf)
        return d if os.path.isdir(d) else None
    except Exception:  # noqa: BLE001 - best effort
        return None


def card_state(dev):
    """current shader / memory clock (the '*' level of pp_dpm_sclk / pp_dpm_mclk), power and edge
    temperature from sysfs, as readable by an ordinary user; None fields when not exposed"""
    out = {"sclk_mhz": None, "mclk_mhz": None, "power_w": None, "temp_c": None}
    d = _pci_dir(dev)
    if d is None:
        return out
    for key, f in (("sclk_mhz", "pp_dpm_sclk"), ("mclk_mhz", "pp_dpm_mclk")):
        try:
            for line in open(os.path.join(d, f)):
                if line.rstrip().endswith("*"):
                    out[key] = int("".join(ch for ch in line.split(":")[1] if ch.isdigit()))
        except (OSError, ValueError, IndexError):
            pass
    try:
        import glob
        for hw in glob.glob(os.path.join(d, "hwmon", "hwmon*")):
            for key, f, scale in (("power_w", "power1_average", 1e-6), ("power_w", "power1_input", 1e-6),
                                  ("temp_c", "temp1_input", 1e-3)):
                fp = os.path.join(hw, f)
                if out[key] is None and os.path.exists(fp):
                    out[key] = round(int(open(fp).read().strip()) * scale, 1)
    except (OSError, ValueError):
        pass
    return out


def card_probe(dev):
    """the card's own speed, to tell a slow box from a code change: a bf16 GEMM (hipBLASLt, 8192^3)
    and a 2 GiB device copy, each timed with HIP events on the current stream"""
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    src = torch.empty(1 << 30, dtype=torch.int16, device=dev).fill_(1)
    dst = torch.empty_like(src)
    res = {}
    for name, fn, work in (("gemm_bf16_tflops", lambda: torch.mm(a, b), 2 * 8192 ** 3 / 1e12),
                           ("hbm_copy_gbs", lambda: dst.copy_(src), 2 * src.numel() * 2 / 1e9)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(work * 10 / (e0.elapsed_time(e1) * 1e-3), 1)
    del a, b, src, dst
    torch.cuda.empty_cache()
    return res


def _spin_rate(dev):
    """torch.cuda._sleep cycles per millisecond on this card (one short calibrated spin)"""
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(20_000_000)
    e1.record()
    torch.cuda.synchronize(dev)
    return 20_000_000 / max(e0.elapsed_time(e1), 1e-3)


def compulsory_bytes(desc):
    """HBM bytes one conv call cannot avoid (bf16): each operand read once, the result written once,
    the weights once; post-op data gradients add their aux reads (post 1/2: the producer's activation,
    post 3: y3 (+ y_ds) + the old gradient + the mask byte, post 4: the mask bits).  The probe's
    descriptor: (kind, N, H, W, C1, C2, K, R, S, stride, pad, ld1, ld2)."""
    kind, N, H, W, C1, C2, K, R, S, stride, pad = desc[:11]
    cin = C1 + C2
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - S) // stride + 1
    mi, mo = N * H * W, N * P * Q
    w = 2 * K * cin * R * S
    if kind.startswith("stem"):
        return N * H * (W + 8) * 16 + w + 2 * mo * K
    if kind.startswith("fwd"):
        return 2 * mi * cin + w + 2 * mo * K
    b = 2 * mo * K + w + 2 * mi * cin  # dgrad: dY, W^T, dX
    if kind.startswith(("dgrad_post1", "dgrad_post2")):
        b += 2 * mi * cin
    elif kind.startswith("dgrad_post3"):
        b += 2 * mi * cin * 2 + mi * cin // 8
    elif kind.startswith("dgrad_post4"):
        b += mi * cin // 8
    return b


def host_enqueue_ms(run, dev, gpu_ms, steps=3):
    """host cost of one step: the GPU is first parked on a spin kernel long enough to cover the
    enqueue, so the launch queue never throttles the host; the wall time of enqueueing `steps` steps
    (the Python op layer and the C-ABI calls of fwd + loss + bwd + Adam), per step.  A step whose
    host cost approaches its GPU time is host-bound: its rate then depends on the box's CPU, not the
    kernels.  Also the host's 1-minute load average, to tell a busy host from a code change."""
    rate = _spin_rate(dev)
    torch.cuda._sleep(int(rate * (steps * max(gpu_ms, 5.0) * 2.5 + 100.0)))
    t0 = time.perf_counter()
    for i in range(steps):
        run(i)
    host = (time.perf_counter() - t0) / steps * 1e3
    torch.cuda.synchronize(dev)
    try:
        load = round(os.getloadavg()[0], 2)
    except OSError:
        load = None
    return round(host, 3), load


def build_step(model_name, batch, size, loss_name, dev, rank, world, args):
    """(model, step fn) of one configuration: synthetic batches resident in HBM, fused Adam with the
    per-bucket overlapped update, the RCCL bucket all-reduce when world > 1"""
    import contextlib

    from model.model_factory import create_model
    from unetseg_hip.arena import FusedAdam
    from unetseg_hip.ddp import GradBuckets
    from unetseg_hip.losses import binary_segmentation_loss, multitask_loss
    from utils.synthetic import make_batch

    torch.manual_seed(11)
    kw = dict(num_classes=1) if model_name == "multitask_unet" else dict(num_classes=2)
    with contextlib.redirect_stdout(sys.stderr):  # weights_init's banner (reference behaviour) -> stderr
        model = create_model(model_name, weights="", **kw).to(dev).train()
    model.compute_dtype = "bf16"
    if world > 1:
        GradBuckets(model, bucket_mb=args.bucket_mb, reduce_dtype=torch.bfloat16 if args.ddp_bf16 else None)
    use_graph = bool(args.graph) and world == 1  # N>1: RCCL collectives stay eager
    overlap = bool(args.overlap_adam) and not use_graph
    opt = FusedAdam(model, lr=1e-4, betas=(0.9, 0.999), weight_decay=1e-4, capturable=use_graph, overlap=overlap,
                    bucket_mb=args.bucket_mb)
    nbatches = 2
    multitask = model_name == "multitask_unet"
    data = []
    for i in range(nbatches):
        x, y, c = make_batch(batch, size, seed=1234 + 100000 * rank + i, with_cls=True)
        data.append((x.to(dev), y.to(dev), c.to(dev)))

    def step(i):
        return step_on(*data[i % nbatches])

    def step_on(x, y, c):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if multitask:  # seg BCE/Lovasz + 1.0 * CE (train.py:213-219 defaults)
                seg, cls = model(x)
                loss = multitask_loss(seg, cls, y, c, 1.0, loss_name)[0]
            else:
                loss = binary_segmentation_loss(model(x), y, loss_name)
        loss.backward()
        opt.step()
        return loss

    run = step
    if args.plan and not use_graph:
        from unetseg_hip.plan import StepPlan
        state = {"plan": None, "eager": 0}

        def run(i):
            p = state["plan"]
            if p is not None:
                x, y, c = data[i % nbatches]
                return p.replay(x=x, y=y, c=c)
            if state["eager"] < 1:  # one eager step first: weights pre-packed, memos and workspaces warm
                state["eager"] += 1
                return step(i)
            x, y, c = data[i % nbatches]
            p = StepPlan({"x": x, "y": y, "c": c})
            loss = p.record(lambda: step_on(x, y, c))  # the recording is a real step
            state["plan"] = p
            return loss
        run.state = state
    if use_graph:
        # one captured step per resident batch; every replay is a full fwd + loss + bwd + Adam step
        # (Adam's lr and step count are device-resident, so replays advance the optimizer state)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for i in range(max(2, args.warmup)):
                step(i)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize()
        graphs = []
        for i in range(nbatches):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                li = step(i)
            graphs.append((gr, li))

        def run(i):
            gr, li = graphs[i % nbatches]
            gr.replay()
            return li
    return model, step, run, use_graph, overlap


def timed(run, steps, warmup, world, dev, sample=None):
    """W untimed steps, then K steps between barrier + synchronize; the wall time is the max over
    ranks.  HIP events between consecutive steps (compute stream: each step ends with the join of
    the weight-gradient stream) give the per-step GPU times for the median."""
    for i in range(warmup):
        run(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    loss = None
    card = None
    for i in range(steps):
        loss = run(i)
        evs[i + 1].record()
        if i == steps // 2 and sample is not None:
            card = sample()  # the host runs ahead of the GPU: this reads the clocks under load
    if sample is not None and card is None:
        card = sample()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    per = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), per[len(per) // 2], evs[0].elapsed_time(evs[-1]), loss, card


#: the other GPU configurations of BASELINE.json, timed in the same process after the headline line
#: (C4 is a one-GPU configuration; C5 is data-parallel, so it runs at every N)
EXTRA = (("c4_attention_unet_b8", "attention_unet", 8, "lovasz_hinge", False),
         ("c5_multitask_unet_b8", "multitask_unet", 8, "bce", True))


def main():
    args = parse()
    from unetseg_hip.ddp import init_from_env, local_device

    rank, world, local = init_from_env("nccl")
    if world != args.gpus:
        if rank == 0:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = torch.device("cuda", local_device(local))
    torch.cuda.set_device(dev)
    torch.manual_seed(11)
    if args.stream:
        # the legacy default stream synchronises implicitly with other streams, which makes the
        # compute stream's final join with the weight-gradient stream slow; work on a created one
        torch.cuda.set_stream(torch.cuda.Stream(dev, priority=args.priority))

    from unetseg_hip import ops

    model, step, run, use_graph, overlap = build_step(args.model, args.batch, args.size, args.loss, dev, rank, world,
                                                      args)
    plan_state = getattr(run, "state", None)
    torch.cuda.reset_peak_memory_stats(dev)
    wall, median_ms, gpu_ms, loss, card_mid = timed(run, args.steps, args.warmup, world, dev,
                                                    sample=lambda: card_state(dev))
    peak_gib = torch.cuda.max_memory_allocated(dev) / 2 ** 30  # caching-allocator peak over warmup + timed steps
    host_ms, host_load = host_enqueue_ms(run, dev, median_ms) if world == 1 and args.host_probe else (None, None)
    ms_per_step = 1000.0 * wall / args.steps
    imgs_per_s = args.batch * world * args.steps / wall
    final_loss = float(loss.item())

    multitask = args.model == "multitask_unet"
    task = "seg+cls multitask" if multitask else "binary seg"
    workload = f"{args.model} {task} {args.size}x{args.size}, per-GPU batch {args.batch}, {args.loss} + Adam"
    roof = None
    if args.probe:
        ops.PROBE = []
        step(0)
        torch.cuda.synchronize()
        kinds = {}
        dump = os.environ.get("UNETSEG_PROBE_DUMP")  # per-call table (kind, desc, us, TFLOP/s)
        if dump:
            with open(dump, "w") as f:
                for kind, flops, nl, e0, e1, desc in ops.PROBE:
                    us = e0.elapsed_time(e1) * 1e3
                    f.write(f"{kind:9s} {us:9.1f} us {flops / max(us, 1e-3) / 1e6:8.1f} TF/s  {desc}\n")
        comp = {}
        floor = {}  # per call max(flops / MFMA peak, compulsory bytes / practical HBM rate), summed
        for kind, flops, nl, e0, e1, desc in ops.PROBE:
            d = kinds.setdefault(kind, [0.0, 0.0, 0])
            d[0] += flops
            d[1] += e0.elapsed_time(e1) * 1e-3
            d[2] += nl
            if desc is not None:
                cb = compulsory_bytes(desc)
                comp[kind] = comp.get(kind, 0) + cb
                floor[kind] = floor.get(kind, 0.0) + max(flops / (PEAK_BF16_TFLOPS * 1e12), cb / HBM_PRACTICAL)
        ops.PROBE = None
        dom = max(kinds, key=lambda k: kinds[k][1])
        fl, sec, n = kinds[dom]
        ach = fl / sec / 1e12
        tr = pmc_traffic(workload, dom)
        mb = pmc_mfma(workload, dom)
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(ach, 2), "peak": PEAK_BF16_TFLOPS,
                "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4), "traffic": tr[0] if tr else None,
                "traffic_unit": "bytes/launch (PMC FETCH_SIZE x2 + WRITE_SIZE)", "traffic_source": tr[1] if tr else None,
                "compulsory_bytes_per_launch": round(comp.get(dom, 0) / n) if n else None,
                "traffic_over_compulsory": round(tr[0] / (comp[dom] / n), 3) if (tr and comp.get(dom) and n) else None,
                "mfma_busy": mb[0] if mb else None, "mfma_busy_source": mb[1] if mb else None,
                "launches_per_step": n, "avg_launch_us": round(1e6 * sec / n, 2),
                "algorithmic_gflop_per_step": round(fl / 1e9, 1),
                "floor_ms_per_step": round(1e3 * floor.get(dom, 0.0), 3),
                "floor_rule": "sum over calls of max(algorithmic flop / MFMA peak, compulsory bytes / 6.3 TB/s)",
                "kernels": {k: {"tflops": round(v[0] / v[1] / 1e12, 2), "ms_per_step": round(1e3 * v[1], 3),
                                "launches": v[2], "floor_ms": round(1e3 * floor.get(k, 0.0), 3)}
                            for k, v in kinds.items()}}

    plan_stats = plan_state["plan"].stats() if plan_state and plan_state["plan"] is not None else None
    # data-parallel consistency: after identical averaged updates every rank holds the same weights
    in_sync = None
    if world > 1:
        cs = model._flat.double().sum().reshape(1)
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        in_sync = bool(float(hi.item()) == float(lo.item()))
    del model, step, run, plan_state
    gc.collect()  # the model and its gradient buckets reference each other
    torch.cuda.empty_cache()

    configs = {}
    if args.extra_configs:
        for tag, name, batch, loss_name, dp in EXTRA:
            if world > 1 and not dp:
                continue
            m2, _, run2, _, _ = build_step(name, batch, args.size, loss_name, dev, rank, world, args)
            ps2 = getattr(run2, "state", None)
            torch.cuda.reset_peak_memory_stats(dev)
            # at least 30 timed steps: a B=8 step is ~10 ms, and over 10 steps one host hiccup of a few
            # ms moved the C5 line by 10-20 % between otherwise identical runs
            k2 = max(args.steps, 30)
            w2, med2, _, _, card2 = timed(run2, k2, args.warmup, world, dev,
                                          sample=(lambda: card_state(dev)) if rank == 0 else None)
            peak2 = torch.cuda.max_memory_allocated(dev) / 2 ** 30
            ips = batch * world * k2 / w2
            host2 = host_enqueue_ms(run2, dev, med2) if world == 1 and args.host_probe else (None, None)
            configs[tag] = {"workload": f"{name} {args.size}x{args.size}, per-GPU batch {batch}, "
                                        f"{loss_name}{' + ce' if name == 'multitask_unet' else ''} + Adam",
                            "value": round(ips, 2), "unit": "images/s", "steps": k2, "ms_per_step": round(1000.0 * w2 / k2, 3),
                            "median_gpu_ms_per_step": round(med2, 3), "peak_alloc_gib": round(peak2, 2),
                            "host_enqueue_ms": host2[0], "host_loadavg": host2[1], "card_during": card2,
                            "step_plan": ps2["plan"].stats() if ps2 and ps2["plan"] is not None else None,
                            "step_mfma_frac": round(ips / world * GFLOP_PER_IMG[name] / 1e3 / PEAK_BF16_TFLOPS, 4)}
            del m2, run2, ps2
            gc.collect()
            torch.cuda.empty_cache()

    card = None
    if rank == 0:
        card = {"during": card_mid, "device": torch.cuda.get_device_name(dev)}
        if args.card_probe:
            card.update(card_probe(dev))

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        cpu = cpu_baseline(args.model, args.size, args.cpu_batch)

    if rank == 0:
        step_tflops = imgs_per_s / world * GFLOP_PER_IMG[args.model] / 1e3
        line = {
            "metric": METRIC, "value": round(imgs_per_s, 2), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (seeded 512x512 RGB ellipse images + masks, resident in HBM)",
            "config": {"workload": workload, "global_batch": args.batch * world,
                       "image_size": args.size, "parallelism": f"dp{world}"},
            "roofline": roof, "cpu_baseline": cpu,
            "step_mfma_frac": round(step_tflops / PEAK_BF16_TFLOPS, 4),
            "step_tflops_per_gpu": round(step_tflops, 2),
            "gpu_event_ms_per_step": round(gpu_ms / args.steps, 3),
            "median_gpu_ms_per_step": round(median_ms, 3), "final_loss": round(final_loss, 5),
            "peak_alloc_gib": round(peak_gib, 2),
            "host_enqueue_ms": host_ms, "host_loadavg": host_load,
            "hip_graph": use_graph, "overlap_adam": overlap, "params_in_sync": in_sync,
            "step_plan": plan_stats,
            "grad_reduce_dtype": ("bf16" if args.ddp_bf16 else "fp32") if world > 1 else None,
            "configs": configs, "card": card,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
