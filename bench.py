#!/usr/bin/env python3
"""Headline benchmark: images/s of the ResNet-50 mixed 8/6/4-bit quantized forward
(BASELINE.json metric; configs[2] at N=1: batch 256 on one MI355X; configs[3] at N=8:
batch 2048 = 8 x 256, weak scaling, RCCL all-gather of logits).

python bench.py --gpus N --steps K --warmup W

N > 1: one process per GPU. Under torch.distributed.run (WORLD_SIZE set) this process is one
rank; started directly with --gpus N it launches `python -m torch.distributed.run
--nproc-per-node N` on itself as a child process before touching the GPU and exits with its code.

One step = one fused forward of 256 synthetic 224x224 images per GPU + the all-gather of the
logits. The inputs are --batches distinct global batches (each rank holds its shard of every
one, generated on device and resident in HBM before the timed region); the first warm-up step
calibrates the static ranges on batch 0, as a real evaluation calibrates on its first batch, and
the timed steps cycle through all of them. Ranks calibrate together (engine.set_dp_group: the
per-layer maxima are MAX-all-reduced), so the gathered logits equal a single-GPU forward of the
global batch bit for bit. Prints ONE
JSON line on rank 0 with the roofline of the dominant kernel family (the quantized conv:
qconv_glds_kernel and the fused stem + pool, every launch incl. the stem) and the CPU baseline (the
reference's fp32 torch-CPU forward restated in oracle/torch_ref.py, timed on a bounded sample).

Timing: `value` comes from the production path, the static-range forward replayed from a
captured HIP graph. HIP events recorded inside a graph capture cannot be timed on ROCm 7.2
(elapsed_time -> hipErrorInvalidHandle, tools/probe_graph_events.py), so the per-launch
kernel durations come from a second region run right after the timed one: the same forward
launched eagerly (the same kernels the graph replays) with HIP events around every conv
launch on the stream it is launched on, one launch at a time (the graph runs each stage's
downsample conv on a side stream beside conv1/conv2; the roofline region runs it serially so
that each event pair times one kernel alone). The roofline is SURVEY.md 8(d)'s: per launch
T_roof = max(2 MACs / P_int8, bytes / BW_HBM) with ops/ops.alg_work's algorithmic bytes.
"""
import argparse
import contextlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(REPO, "semilayer-wise-mixed-precision-quantization_amd")
for _p in (PKG_DIR, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec ResNet-50 mixed 8/6/4b @224×224, 1/2/4/8 MI355X; % int8 roofline"
# MI355X dense int8 MFMA peak: v_mfma_i32_16x16x64_i8 = 2x the bf16 rate (MI355X_MICROARCH.md
# 'Matrix cores': I8 row), bf16 dense ~2.5 PF  ->  ~5.0 POPS dense (no sparsity).
INT8_DENSE_PEAK_TOPS = 5000.0
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    "r50_mixed": ("resnet50", "r50_mixed", "ResNet-50 mixed 8/6/4-bit (published semilayer assignment), 224x224"),
    "r18_u8": ("resnet18", "r18_u8", "ResNet-18 uniform int8 addressable convs, 224x224"),
    "r34_4bit": ("resnet34", "r34_4bit", "ResNet-34 4-bit-dominant semilayer mix, 224x224"),
}


class ConvTimer:
    """HIP events around every quantized-conv launch, on the stream it is launched on."""

    def __init__(self):
        self.recs = []
        self.active = False
        self._ev = None

    def begin(self):
        if self.active:
            self._ev = torch.cuda.Event(enable_timing=True)
            self._ev.record(torch.cuda.current_stream())

    def end(self, work):
        if self.active:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(torch.cuda.current_stream())
            self.recs.append((self._ev, e1, work))

    def print_layers(self, steps):
        """Per-launch table of the last step: time, floor T_roof and the dominant resource."""
        n = len(self.recs) // max(steps, 1)
        rows = []
        for a, b, w in self.recs[-n:]:
            t = a.elapsed_time(b) * 1e-3
            tm = w["ops"] / (INT8_DENSE_PEAK_TOPS * 1e12)
            th = w["bytes"] / (HBM_PEAK_GBS * 1e9)
            rows.append((w.get("shape", "?"), t, tm, th, w["passes"]))
        print("%-28s %9s %9s %9s %6s %8s %8s" % ("launch", "t_us", "mfma_us", "hbm_us", "roof", "TOP/s", "GB/s"),
              file=sys.stderr)
        for sh, t, tm, th, p in rows:
            print("%-28s %9.1f %9.1f %9.1f %6.3f %8.1f %8.1f" % (sh, t * 1e6, tm * 1e6, th * 1e6, max(tm, th) / t,
                                                            tm * INT8_DENSE_PEAK_TOPS / t, th * HBM_PEAK_GBS / t),
                  file=sys.stderr)
        tt = sum(r[1] for r in rows)
        print("total %.1f us, floor %.1f us" % (tt * 1e6, sum(max(r[2], r[3]) for r in rows) * 1e6), file=sys.stderr)

    def roofline(self, steps):
        """per launch T_roof = max(ops / P_int8, bytes / BW); the reported
        bound is the resource whose floor dominates the sum."""
        torch.cuda.synchronize()
        t = [a.elapsed_time(b) * 1e-3 for a, b, _ in self.recs]
        w = [r[2] for r in self.recs]
        n = len(t)
        t_sum = sum(t)
        ops = sum(x["ops"] for x in w)
        nbytes = sum(x["bytes"] for x in w)
        pass_ops = sum(x["ops"] * x["passes"] for x in w)
        t_mfma = ops / (INT8_DENSE_PEAK_TOPS * 1e12)
        t_hbm = nbytes / (HBM_PEAK_GBS * 1e9)
        t_roof = sum(max(x["ops"] / (INT8_DENSE_PEAK_TOPS * 1e12), x["bytes"] / (HBM_PEAK_GBS * 1e9)) for x in w)
        hbm_gbs = nbytes / t_sum / 1e9
        tops = ops / t_sum / 1e12
        if t_hbm >= t_mfma:
            bound, achieved, peak, unit = "hbm", hbm_gbs, HBM_PEAK_GBS, "GB/s"
        else:
            bound, achieved, peak, unit = "mfma", tops, INT8_DENSE_PEAK_TOPS, "TFLOP/s"
        return {
            "bound": bound, "achieved": round(achieved, 2), "peak": peak, "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": None,
            "kernel": "quantized conv (qconv_glds_kernel + qconv_halo_kernel + qconv_stem_pool_kernel), all launches incl. the stem",
            "launches_per_step": n // max(steps, 1),
            "avg_launch_ms": round(t_sum / max(n, 1) * 1e3, 5),
            "alg_bytes_per_launch": round(nbytes / max(n, 1)),
            "alg_ops_per_launch": round(ops / max(n, 1)),
            "t_roof_over_t": round(t_roof / t_sum, 4),
            "hbm_frac": round(hbm_gbs / HBM_PEAK_GBS, 4),
            "mfma_frac": round(tops / INT8_DENSE_PEAK_TOPS, 4),
            "mfma_frac_incl_limb_passes": round(pass_ops / t_sum / 1e12 / INT8_DENSE_PEAK_TOPS, 4),
            "conv_ms_per_step": round(t_sum / max(steps, 1) * 1e3, 4),
            "timing": "HIP events per launch over %d eager steps right after the graph-replayed timed "
                      "region (same kernels; events cannot time inside a replayed HIP graph)" % steps,
        }


def attach_traffic(roof, config, limbs, batch, streams):
    """roofline.traffic: HBM bytes per quantized-conv launch from the committed PMC measurement of
    this workload (tools/pmc_traffic.sh: FETCH_SIZE and WRITE_SIZE passes of rocprofv3 over this
    bench's eager roofline region, gfx950-corrected by tools/pmc_traffic.py). PMC counters cannot
    be read from inside a normal run, so the number comes from that profile. It is attached only
    when the profile was taken on this very library (build stamp), tile table (content hash) and
    launch layout; otherwise traffic is null and roofline.traffic_note says why."""
    path = os.path.join(REPO, "profiles", "pmc_traffic_%s_L%d_B%d_S%d.json" % (config, limbs, batch, streams))
    if not os.path.exists(path):
        roof["traffic_note"] = "no PMC profile " + os.path.relpath(path, REPO)
        return
    m = json.load(open(path))
    from smpq import _lib, ops
    stamp = _lib.load().smpq_build_stamp().decode()
    why = []
    if m.get("lib_stamp") != stamp:
        why.append("library build stamp %s != %s" % (str(m.get("lib_stamp"))[:16], stamp[:16]))
    if m.get("tile_table_sha16") != ops.tile_table_info()["sha16"]:
        why.append("tile table %s != %s" % (m.get("tile_table_sha16"), ops.tile_table_info()["sha16"]))
    if m.get("launches") != roof["launches_per_step"] * m.get("rsteps", 3):
        why.append("launches %s != %d" % (m.get("launches"), roof["launches_per_step"] * m.get("rsteps", 3)))
    if why:
        roof["traffic_note"] = "stale PMC profile (%s): %s" % (os.path.basename(path), "; ".join(why))
        return
    roof["traffic"] = m["traffic_bytes_per_launch"]
    roof["traffic_over_alg_bytes"] = round(m["traffic_bytes_per_launch"] / roof["alg_bytes_per_launch"], 4)
    roof["traffic_source"] = "profiles/" + os.path.basename(path) + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE)"


def _cpu_model():
    """The host CPU's model name (/proc/cpuinfo), or the platform's processor string."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(arch, assign_name, batch, iters=2):
    """the reference CPU path (the fp32 torch forward of oracle/torch_ref.py, the
    reference's own operators, on the weights fake-quantized by the oracle quantizer — bit-exact
    with functions.channel_wise_quantizationperchan) at the config's batch: 1 warm-up and ``iters``
    timed iterations of one [batch, 3, 224, 224] N(0,1) batch (seed 1), all of torch's CPU threads
    (OMP_NUM_THREADS: the box's CPU share), the host CPU model recorded."""
    from oracle import quant_ref, torch_ref
    import resnet
    from smpq import assignments
    torch.manual_seed(0)
    net = getattr(resnet, arch)()
    sd = {k: v.clone() for k, v in net.state_dict().items() if not k.endswith(("qbits", "qstep"))}
    asg = assignments.load_assignment(assign_name)
    names = {id(m): n for n, m in net.named_modules()}
    for ln, cn, ch in zip(asg["lnum"], asg["cnum"], asg["chain"]):
        key = names[id(assignments.conv_for_lnum(net, int(ln)))] + ".weight"
        sd[key][cn] = torch.from_numpy(quant_ref.apply_chain(sd[key][cn].numpy(), [int(b) for b in ch if b]))
    threads = torch.get_num_threads()
    x = torch.randn(batch, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    t0 = time.perf_counter()
    torch_ref.resnet_forward(arch, sd, x)  # warm-up (one full batch)
    warm = time.perf_counter() - t0
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        torch_ref.resnet_forward(arch, sd, x)
        ts.append(time.perf_counter() - t0)
    el = sum(ts)
    return {"value": round(batch * iters / el, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": "the fp32 torch-CPU reference forward of %s on the same fake-quantized weights, batch %d, "
                      "1 warm-up (%.2f s) + %d timed iterations (%s s), %d torch threads on %s"
                      % (arch, batch, warm, iters, "/".join("%.2f" % t for t in ts), threads, _cpu_model())}


# the int8-fused roofline of the quantized convs (int8 activations between convs,
# BN / ReLU / residual fused), per config at the batch it is quoted for, ms
INT8_FUSED_FLOOR_MS = {"r50_mixed": (256, 0.666), "r18_u8": (256, 0.179), "r34_4bit": (512, 0.742)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 100 timed steps after 20 warm-up steps (~1 s of GPU time): a steady-state rate
    # (20 / 5 read 1-2 % lower on the same box, profiles/r06_bench_length.txt)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU per step")
    ap.add_argument("--config", default="r50_mixed", choices=sorted(CONFIGS))
    ap.add_argument("--limbs", type=int, default=3,
                    help="activation int8 limbs: 3 = int24 codes (parity mode, default), 2 = int16 (fast mode)")
    ap.add_argument("--roofline-steps", type=int, default=3, help="eager steps timed per launch for the roofline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--layers", action="store_true", help="print a per-launch roofline table (stderr)")
    ap.add_argument("--cpu-iters", type=int, default=2, help="timed CPU-baseline iterations (after 1 warm-up)")
    ap.add_argument("--chunk", type=int, default=None, help="images per pass (Infinity-Cache blocking)")
    ap.add_argument("--streams", type=int, default=None,
                    help="batch slices run concurrently on their own streams (default: engine.STREAMS)")
    ap.add_argument("--batches", type=int, default=4,
                    help="distinct device-resident global batches cycled through the timed steps")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: relaunch under torch.distributed.run as a CHILD (no exec), before
        # this process touches the GPU
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import __graft_entry__
    if rank == 0 or world == 1:
        __graft_entry__.build()
    if world > 1:
        dist.barrier()
        __graft_entry__.build()
    import resnet
    from smpq import assignments, dp, ops, stats

    arch, assign, desc = CONFIGS[args.config]
    ops.set_act_limbs(args.limbs)
    from smpq import engine
    if args.chunk:
        engine.set_chunk(args.chunk)
    if args.streams:
        engine.STREAMS[0] = args.streams
    # every step below runs on every rank in lockstep: the ranks calibrate together (MAX-all-reduced
    # maxima) for as long as the block lasts (dp.lockstep scopes the engine's group to it)
    lockstep = contextlib.ExitStack()
    lockstep.enter_context(dp.lockstep())
    torch.manual_seed(0)
    net = getattr(resnet, arch)().to(dev).eval()
    assignments.apply_assignment(net, assign)

    # this rank's shard of every global batch (dp.shard_range), generated on device; the seed
    # depends on the batch and the shard's first image only
    s0, s1 = dp.shard_range(args.batch * world, rank, world)
    xs = []
    # every batch gets its graph (captured on its own input memory) within the W warm-up steps:
    # the first warm-up step calibrates, each further one captures one batch's graph
    nb = max(1, min(args.batches, args.warmup - 1)) if args.warmup > 1 else 1
    for b in range(nb):
        g = torch.Generator(device=dev).manual_seed(1000 + 1000003 * b + s0)
        xs.append(torch.randn(s1 - s0, 3, 224, 224, generator=g, device=dev))
    gathered = torch.empty(world * args.batch, 1000, device=dev) if world > 1 else None
    it = [0]

    def step():
        x = xs[it[0] % len(xs)]
        it[0] += 1
        with torch.no_grad():
            y = net(x)
            return dp.gather_logits(y, world, out=gathered)

    for _ in range(max(1, args.warmup)):
        step()  # the first one calibrates on batch 0
    if rank == 0:
        print("tiles (%s):" % json.dumps(ops.tile_table_info()),
              {ops.key_str(k): v for k, v in ops._TUNED.items()}, file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    st0 = {k: stats[k] for k in ("calibrations", "overflow_reruns", "stale_reruns", "graph_captures")}
    # HIP events around every step on the stream the graph is replayed on: the GPU time of the
    # timed region itself (both batch slices concurrent), the roofline's per-launch time
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record()
        step()
        e1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    gpu_ms_timed = sum(e0.elapsed_time(e1) for e0, e1 in evs)
    timed_stats = {k: stats[k] - v for k, v in st0.items()}
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    # per-launch kernel durations for the roofline: the same forward, launched eagerly, one launch
    # at a time (events time each kernel alone). Region 1: the whole batch per launch (for
    # reference); region 2 (last, so that tools/pmc_traffic.sh's PMC passes see it as the last
    # dispatches): the timed path's own batch slices and tile choices, the slices run one after
    # the other on one stream. The roofline line reports region 2.
    use_graph, conc, nst = engine.USE_GRAPH[0], engine.CONCURRENT_DS[0], engine.STREAMS[0]

    def eager_region(streams):
        timer = ConvTimer()
        engine.USE_GRAPH[0] = False
        engine.CONCURRENT_DS[0] = False
        engine.STREAMS[0] = streams
        engine.SERIAL_SLICES[0] = True
        ops.set_conv_hook(timer)
        step()  # untimed: the eager path's first pass
        timer.active = True
        for _ in range(args.roofline_steps):
            step()
        timer.active = False
        ops.set_conv_hook(None)
        engine.USE_GRAPH[0], engine.CONCURRENT_DS[0], engine.STREAMS[0] = use_graph, conc, nst
        engine.SERIAL_SLICES[0] = False
        return timer

    sliced = nst > 1 and args.batch >= 2 * nst
    whole = eager_region(1) if sliced else None
    timer = eager_region(nst)
    lockstep.close()
    iso = timer.roofline(args.roofline_steps)
    images = args.batch * world * args.steps
    value = images / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    # The roofline of the timed region: its per-launch time = the event-timed GPU time of a step
    # divided by the step's launches (the two batch slices run concurrently, so a launch's share of
    # the step, not its isolated duration, is what the throughput is made of); its algorithmic
    # bytes and ops per launch are those of the same launches (the isolated region below runs the
    # same kernels one at a time).
    n_l = iso["launches_per_step"]
    step_gpu_ms = gpu_ms_timed / args.steps
    t_launch = step_gpu_ms / n_l * 1e-3
    hbm_gbs = iso["alg_bytes_per_launch"] / t_launch / 1e9
    tops = iso["alg_ops_per_launch"] / t_launch / 1e12
    roof = {"bound": iso["bound"], "achieved": round(hbm_gbs if iso["bound"] == "hbm" else tops, 2),
            "peak": iso["peak"], "unit": iso["unit"],
            "frac": round((hbm_gbs / HBM_PEAK_GBS) if iso["bound"] == "hbm" else (tops / INT8_DENSE_PEAK_TOPS), 4),
            "traffic": None, "kernel": iso["kernel"], "launches_per_step": n_l,
            "avg_launch_ms": round(t_launch * 1e3, 5),
            "alg_bytes_per_launch": iso["alg_bytes_per_launch"], "alg_ops_per_launch": iso["alg_ops_per_launch"],
            "hbm_frac": round(hbm_gbs / HBM_PEAK_GBS, 4), "mfma_frac": round(tops / INT8_DENSE_PEAK_TOPS, 4),
            "mfma_frac_incl_limb_passes": round(iso["mfma_frac_incl_limb_passes"] * iso["avg_launch_ms"] / (t_launch * 1e3), 4),
            "gpu_ms_per_step": round(step_gpu_ms, 4),
            "kernel_share_of_step": round(step_gpu_ms / ms_per_step, 4),
            "timing": "HIP events around each of the %d timed steps (graph replays) on their stream: the step's GPU "
                      "time / its %d quantized-conv launches (non-conv kernels of the step included in the time)"
                      % (args.steps, n_l)}
    iso["region"] = ("the timed path's %d batch slices of %d images per launch and its tile choices, one launch at "
                     "a time" % (nst, -(-args.batch // nst))) if sliced else \
        "the whole batch of %d images per launch, one launch at a time" % args.batch
    roof["isolated"] = {k: iso[k] for k in ("frac", "achieved", "avg_launch_ms", "conv_ms_per_step", "t_roof_over_t",
                                            "mfma_frac_incl_limb_passes", "timing", "region")}
    if whole is not None:
        rw = whole.roofline(args.roofline_steps)
        roof["whole_batch"] = {k: rw[k] for k in ("frac", "achieved", "avg_launch_ms", "launches_per_step",
                                                   "conv_ms_per_step", "mfma_frac_incl_limb_passes")}
        roof["whole_batch"]["region"] = "the whole batch of %d images per launch, one launch at a time" % args.batch
    if args.layers and rank == 0:
        (whole or timer).print_layers(args.roofline_steps)
    attach_traffic(roof, args.config, args.limbs, args.batch, nst if sliced else 1)
    # how far the north star is: BASELINE.md's int8-fused floor of this config (1-byte activations
    # between the quantized convs) over the measured step, beside the 3-byte-format frac above
    fb, fms = INT8_FUSED_FLOOR_MS[args.config]
    roof["int8_fused_floor_ms"] = round(fms * args.batch / fb, 4)
    roof["int8_fused_frac"] = round(roof["int8_fused_floor_ms"] / ms_per_step, 4)
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "i8",
            "data": "synthetic (N(0,1) 224x224 on device; seeded random-init weights, reference init)",
            "config": {"workload": desc, "assignment": assign, "batch_per_gpu": args.batch,
                       "global_batch": args.batch * world, "act_limbs": args.limbs,
                       "act_code": {1: "int8", 2: "int16 (2 int8 limbs)", 3: "int24 (3 int8 limbs)"}[args.limbs],
                       "parallelism": "dp%d" % world, "quantized_convs_per_step": roof["launches_per_step"],
                       "range_mode": engine.get_range_mode(), "chunk": engine.CHUNK[0],
                       "hip_graph": bool(engine.USE_GRAPH[0]),
                       "concurrent_downsample": bool(engine.CONCURRENT_DS[0]),
                       "batch_slices_on_streams": engine.STREAMS[0],
                       "distinct_batches": len(xs),
                       "calibrations_total": stats["calibrations"],
                       "timed_calibrations": timed_stats["calibrations"],
                       "timed_overflow_reruns": timed_stats["overflow_reruns"],
                       "timed_stale_reruns": timed_stats["stale_reruns"],
                       "timed_graph_captures": timed_stats["graph_captures"],
                       "tile_table": ops.tile_table_info()},
            "roofline": roof,
        }
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(arch, assign, args.batch, args.cpu_iters)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
