"""Throughput of the MI355X Sep-TFAnet^VAD forward path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--precision f16x3|fp32|bf16|f16]
                    [--workload offline|cfg4|cfg5|long|stream]

One step = one ``SeparationModel.forward`` (config_with_vad.json) over a resident batch of 64
synthetic 2-speaker mixtures of 32 000 samples (4 s @ 8 kHz resampled to 16 kHz by the
reference's CLI, only_inference.py:76-79 => T = 126 frames) per GPU. One process per GPU: the
driver launches the ranks with torch.distributed.run; ``--gpus N`` without a torchrun environment
starts them itself (a child torch.distributed.run, before this process touches the GPU). Every rank
runs its own shard of utterances (weak scaling, no collective on the data path, only barriers around
the timed region and a max-reduce of the elapsed time). Rank 0 prints one JSON line.

Extra fields:
  roofline      (+ weight_stream: the per-CU weight bytes of the launch, their rate, and the texture-path
                busy fraction from the committed counters — the decomposition's real floor)
                dominant kernel = k_tcn, the fused persistent TCN (24 blocks of conv1d 256->256, depthwise
                conv, res_out 512->256, TF-attention, recursive LN in one launch); algorithmic FLOPs per
                launch (its two pointwise GEMMs per block) / its average launch time from HIP events that
                libsepvad records on the stream the kernel runs on. On the multi-kernel
                schedule (fp32 GEMMs, T > 1024, SEPVAD_FUSED=0) the res_out GEMM.
  cpu_baseline  the oracle CPU restatement (oracle/torch_ref.py, torch fp32) on every core of this
                process's CPU share (the cgroup quota caps it: 16 on the GPU box, where os.cpu_count()
                reports the whole machine), rank 0 at N=1 only, on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "utterances/sec/GPU (4s@8kHz, 2spk+VAD); SI-SDR within 0.01 dB of ref"
B_PER_GPU = 64
N_SAMPLES = 32000
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: F32 matrix (= vector) peak, dense
F16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: BF16/F16 dense MFMA peak (no sparsity)
HBM_PEAK_GBS = 8000.0


def gemm_flops_per_utt(T):
    """Algorithmic FLOPs of the 1x1 GEMMs per utterance: 9 700 352 * T."""
    return (24 * (2 * 256 * 256 + 2 * 512 * 256) + 2 * 514 * 256) * T


def res_out_flops(B, T):
    return 2 * 256 * 512 * B * T


def tcn_flops(B, T, precision="f16x3", nblk=24):
    """Algorithmic FLOPs of one fused-TCN launch: the two pointwise GEMMs of every block and the output head that
    runs inside the launch since round 4 (SURVEY §8d F_gemm): (24 * 2 * (256*256 + 512*256) + 2 * 514 * 256) per
    frame."""
    return (nblk * 2 * (256 * 256 + 512 * 256) + 2 * 514 * 256) * B * T


def weight_bytes(precision, wlo="f16"):
    """Bytes per pointwise weight streamed by the fused TCN: fp16 hi + fp16 lo (f16x3), fp16 hi + a byte lo plane
    (f16x3 with --wlo e4m3 / i8), one 16-bit plane (f16 / bf16) or fp32."""
    if precision == "fp32":
        return 4
    return (4 if wlo == "f16" else 3) if precision == "f16x3" else 2


HEAD_ROWS_MFMA = 512  # output-head rows on MFMA inside k_tcn (bins 0..255 of 2 speakers; bin 256 on VALU)


def tcn_bytes(B, T, precision="f16x3", wlo="f16"):
    """Compulsory HBM bytes of one fused-TCN launch: TCN input read (fp32 [B][Tp][256]), the head's masks written
    (fp32, 514 of [B][Tp][576]) and its VAD tap products ([B][2][Tp][20]), the weights in fragment order read once
    (24 blocks x 768 KB as fp16 hi/lo, 576 KB with a byte lo plane, 384 KB as one 16-bit plane; the head's 512 MFMA
    rows likewise)."""
    Tp = (T + 31) // 32 * 32
    wbytes = weight_bytes(precision, wlo)
    return (B * Tp * 256 * 4 + B * Tp * 514 * 4 + B * 2 * Tp * 20 * 4
            + (24 * (256 * 256 + 256 * 512) + HEAD_ROWS_MFMA * 256) * wbytes)


TA_FILE = "r06prof_pmc_ta_summary.txt"  # texture-path counters of k_tcn (tools/r05_profile.sh), cfg 2, f16x3, i8 lo
CACHE_FILE = "r06prof_coexec_tcc_dram.txt"  # MFMA/VALU co-issue, L2 hit/miss and memory-side read counters
RING_FILE = "r02bi_ring_gemm.txt"       # GEMM-phase stream floor per CU (tools/probe_src/ring_gemm.hip)
STREAM_FLOOR_GBPS = 103.2


def weight_stream(B, T, precision, avg_launch_s, n_cu=256, wlo="f16", nsl=1):
    """The fused TCN's per-CU weight stream: every workgroup pulls every block's weights once per utterance it
    runs, for its nsl 32-frame slices together, so each CU moves rounds x 24 x (256x256 + 512x256)
    x 4 (fp16 hi/lo), 3 (byte lo plane) or 2 bytes per launch. With the texture-path busy fraction from the committed
    counters where they apply."""
    G = (T + 31) // 32
    slices = -(-B * (G // nsl) // n_cu)
    wbytes = weight_bytes(precision, wlo)
    per_cu = slices * 24 * (256 * 256 + 256 * 512) * wbytes
    rate = per_cu / avg_launch_s / 1e9
    out = {"bytes_per_cu_per_launch": per_cu, "workgroup_rounds": slices, "slices_per_workgroup": nsl, "achieved_GBps_per_cu": round(rate, 2),
           # the same two GEMMs streamed back to back with nothing else (tools/probe_src/ring_gemm.hip)
           "floor_GBps_per_cu": STREAM_FLOOR_GBPS, "frac_of_floor": round(rate / STREAM_FLOOR_GBPS, 3),
           "floor_source": "profiles/" + RING_FILE, "ta_busy_frac": None, "ta_source": None}
    path = os.path.join(REPO, "profiles", TA_FILE)
    if precision == "f16x3" and wlo == PMC_WLO and B == B_PER_GPU and T == 1 + N_SAMPLES // 256 and os.path.exists(path):
        try:
            lines = open(path).read().splitlines()
            i = next(k for k, ln in enumerate(lines) if "k_tcn" in ln)
            kv = dict(t.split("=") for t in lines[i + 1].split())
            out["ta_busy_frac"] = round(float(kv["TA_BUSY_avr"]) / (float(kv["GRBM_GUI_ACTIVE"]) / 8), 3)
            out["ta_source"] = "profiles/" + TA_FILE + " (TA_BUSY_avr per CU / GRBM_GUI_ACTIVE per XCD)"
        except (OSError, StopIteration, KeyError, ValueError):
            pass
    return out


def cache_counters(wlo):
    """k_tcn's L2 hit rate, MFMA/VALU co-issue and the attribution of `traffic` from the committed counter passes
    (profiles/CACHE_FILE, headline configuration). The L2's memory-side reads count as DRAM-bound whether the
    Infinity Cache serves them or not (TCC_EA0_RDREQ_DRAM_sum == TCC_EA0_RDREQ_sum), so the IC / HBM split is a
    model: every XCD's L2 fetches each block's weights once (the weights stay IC-resident: 19.3 MB of 256 MB)."""
    out = {"source": "profiles/" + CACHE_FILE}
    try:
        lines = open(os.path.join(REPO, "profiles", CACHE_FILE)).read().splitlines()
        vals = {}
        for i, ln in enumerate(lines):
            if "k_tcn" in ln and i + 1 < len(lines):
                vals.update(dict(t.split("=") for t in lines[i + 1].split()))
        hit, miss = float(vals["TCC_HIT_sum"]), float(vals["TCC_MISS_sum"])
        out["l2_hit_rate"] = round(hit / (hit + miss), 4)
        out["mfma_busy_coissued_with_valu"] = round(float(vals["SQ_VALU_MFMA_COEXEC_CYCLES"])
                                                    / float(vals["SQ_VALU_MFMA_BUSY_CYCLES"]), 3)
        out["dram_bound_share_of_l2_reads"] = round(float(vals["TCC_EA0_RDREQ_DRAM_sum"])
                                                    / float(vals["TCC_EA0_RDREQ_sum"]), 3)
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        pass
    w = (24 * (256 * 256 + 256 * 512) + HEAD_ROWS_MFMA * 256) * weight_bytes("f16x3", wlo)
    out["weights_bytes"] = w
    out["model"] = {"per_xcd_weight_fetch_bytes": 8 * w, "ic_served_upper_bound_bytes": 7 * w,
                    "note": "8 XCD L2s each fetch the launch's weights once; all but one copy can come from the "
                            "Infinity Cache (upper bound on IC-served bytes); the rest of `traffic` is activations "
                            "and hand-off words"}
    return out


def res_out_bytes(B, T):
    """Compulsory bytes of one res_out launch: operand d as fp16 hi+lo planes (B*Tp x 512 x 4 B),
    output r fp32 (B*Tp x 256 x 4 B), fp16 hi/lo weights (256 x 512 x 4 B)."""
    Tp = (T + 63) // 64 * 64
    return B * Tp * 512 * 4 + B * Tp * 256 * 4 + 256 * 512 * 4


STATS_FILE = "r06prof_kernel_stats.csv"  # rocprofv3 --kernel-trace --stats of the headline bench command (cfg 2, f16x3)
TCN_KERNEL_PREFIX = "void sepvad::k_tcn<2, 1, false, 2, false, false, 1>"  # the dominant kernel's name in that file


def rocprof_avg_us(kernel_prefix):
    """Average duration (us) of the kernel whose name starts with `kernel_prefix` in the committed rocprofv3 stats of
    the headline command (profiles/STATS_FILE), so the roofline fraction is reproducible from profiles/ alone."""
    import csv
    path = os.path.join(REPO, "profiles", STATS_FILE)
    try:
        for r in csv.DictReader(open(path)):
            if r["Name"].startswith(kernel_prefix):
                return float(r["AverageNs"]) / 1e3
    except (OSError, KeyError, ValueError):
        pass
    return None


PMC_FILE = "r01h_pmc_res_out.json"       # multi-kernel schedule (res_out GEMM)
PMC_FILE_FUSED = "r06prof_pmc_tcn.json"     # fused schedule (k_tcn)
PMC_WLO = "i8"                             # ... measured with this weight lo plane
DEFAULT_SPLIT = 1
# Default (timed steps, warmup steps) per workload: ~0.1 s of untimed load, then ~0.5 s timed. The shader clock ramps
# during the first tens of milliseconds of load: 3 warmup steps and 20 timed ones (rounds 1-5) measured the ramp,
# 122-124k utt/s at cfg 2 against 137-140k with 100+ warmup steps on the same box (profiles/r05_warm/lines.txt).
STEADY_STEPS = {"offline": (1000, 200), "cfg4": (600, 120), "cfg5": (600, 120), "long": (600, 120), "stream": (40, 8)}


def host_cores():
    """CPU cores this process may use: the affinity set, capped by the cgroup CPU quota. On the GPU box
    os.cpu_count() reports the whole machine while the job's share is 16 CPUs; threading to the machine
    count there oversubscribes the share many times over."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(seconds: float = 12.0):
    """Oracle (CPU restatement, torch fp32) on the host: batches of the same workload until
    `seconds` of CPU work have elapsed (at least 2 batches)."""
    from oracle.torch_ref import OracleModel
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    threads = host_cores()  # every core of this process's CPU share, stated in the line
    torch.set_num_threads(threads)
    sd = {k: torch.from_numpy(v) for k, v in synth.make_state_dict(pkg.CONFIG_WITH_VAD, 1234).items()}
    om = OracleModel(pkg.CONFIG_WITH_VAD, sd, torch.float32)
    x, _ = synth.make_batch(B_PER_GPU, N_SAMPLES, 7000)
    xt = torch.from_numpy(x)
    om(xt[:2])  # warm-up
    n_utt, t0 = 0, time.perf_counter()
    while True:
        om(xt)
        n_utt += B_PER_GPU
        el = time.perf_counter() - t0
        print(f"cpu_baseline: {n_utt} utterances in {el:.1f} s", file=sys.stderr, flush=True)
        if el >= seconds and n_utt >= 2 * B_PER_GPU:
            break
    return dict(value=n_utt / el, unit="utterances/s", cores=threads, kind="port",
                sample=f"{n_utt} utterances ({n_utt // B_PER_GPU} batches of B={B_PER_GPU}, N={N_SAMPLES}) "
                       f"in {el:.1f} s, oracle/torch_ref.py fp32 on {threads} threads (this process's CPU share: "
                       f"affinity capped by the cgroup quota; os.cpu_count() = {os.cpu_count()})")


_JSON_FD = None


def hold_stdout():
    """From here on the process's fd 1 is its stderr; only emit() writes to the real stdout. Native libraries
    print banners to fd 1 (RCCL prints its version / hostname at init on some hosts), and the driver reads
    exactly one JSON line from rank 0's stdout."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def emit(obj):
    line = (json.dumps(obj) + "\n").encode()
    sys.stdout.flush()
    if _JSON_FD is None:
        os.write(1, line)
    else:
        os.write(_JSON_FD, line)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """``--gpus N`` (N > 1) outside a torchrun environment: run N ranks, one process per GPU, as a child
    ``torch.distributed.run`` and return its exit code. Called before anything touches the GPU (this
    process never initialises HIP, so nothing is exec'd from a GPU process). None = run in-process."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def init_dist(args, backend="nccl"):
    """(dist or None, world, rank, local_rank) of this rank; world must equal --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    d = None
    # SEPVAD_BENCH_SHARE_GPU=1 (tests only): every rank on cuda:0 with a gloo process group, so the N-rank launcher,
    # the barrier / max-reduce and the stream PIT all-reduce run end to end on a one-GPU box (RCCL needs a GPU per
    # rank); timing from this mode is not a scaling measurement
    if os.environ.get("SEPVAD_BENCH_SHARE_GPU") == "1":
        backend, local_rank = "gloo", 0
    # SEPVAD_BENCH_FORCE_DIST=1: the process group even at world 1 (exercises the RCCL barrier / max-reduce
    # path of the timed region on a one-GPU box)
    if world > 1 or os.environ.get("SEPVAD_BENCH_FORCE_DIST") == "1":
        import torch.distributed as d
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            d.init_process_group(backend, device_id=torch.device("cuda", local_rank))
        else:
            d.init_process_group(backend)
    return d, world, rank, local_rank


def _reduce_dev(dist, dev):
    """Device of the max-over-ranks reduction: the GPU under RCCL, the host under gloo."""
    return "cpu" if dist is not None and dist.get_backend() == "gloo" else dev


def timed_region(step, steps, warmup, dist=None, sync=lambda: None, reduce_device="cpu"):
    """W untimed warmup steps, then EXACTLY `steps` steps bracketed by a barrier + device sync on both
    sides; returns the elapsed seconds, max over ranks (the driver contract)."""
    for _ in range(warmup):
        step()
    sync()

    def barrier():
        if dist is not None:
            dist.barrier()
        sync()

    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], device=reduce_device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def bench_stream(args):
    """BASELINE cfg 3: OnlineSaving (model/online_class_unknown_targets.py:72-105) over 256 streams of
    4 s @ 16 kHz, 3 s windows at a 160 ms hop (7 windows per stream, each a batched B=256 forward of
    48 000 samples, T=188), PIT-L1 realignment and stitching on the device. One step = one calc_online
    over all streams. value = stream-windows/s (whole job); audio_seconds_per_second = value * save_sec
    (seconds of new audio emitted per wall-clock second, all streams together)."""
    dist, world, rank, local_rank = init_dist(args)
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    import contextlib
    import io
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    cfg = pkg.CONFIG_WITH_VAD
    with contextlib.redirect_stdout(io.StringIO()):
        net = pkg.SeparationModel(**cfg)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.make_state_dict(cfg, 1234).items()}, strict=True)
    net = net.eval().to(dev)
    n_streams, n_total, save_sec = args.batch or 256, 64000, 0.16
    x = torch.from_numpy(synth.make_batch(n_streams, n_total, 20_000 + rank * n_streams)[0]).to(dev)
    net.native_handle(dev).reserve(n_streams, 48000)
    crit = pkg.PITLossWrapper(loss_func=torch.nn.L1Loss(), pit_from="pw_pt")
    ons = pkg.OnlineSaving(net, "/nonexistent", crit)
    ons.save_sec = save_sec
    n_win = ons.n_windows(n_total)
    ikw = dict(pkg.INFERENCE_KW_DEFAULTS)

    group = dist.group.WORLD if dist is not None else None

    def step():
        ons.calc_online(x, "bench", 10 ** 6, ikw, process_group=group)

    el = timed_region(step, args.steps, args.warmup, dist, torch.cuda.synchronize, _reduce_dev(dist, dev))
    if os.environ.get("SEPVAD_BENCH_DUMP"):  # tests: this rank's stitched streams after the last step
        np.save(f"{os.environ['SEPVAD_BENCH_DUMP']}.rank{rank}.npy", ons.online_signal.cpu().numpy())
    if rank == 0:
        windows = world * n_streams * n_win * args.steps
        out = {
            "metric": "stream-windows/sec (cfg 3: OnlineSaving, 3 s windows, 160 ms hop, PIT-L1 stitching)",
            "value": round(windows / el, 2), "unit": "windows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic PCG64 mixtures",
            "config": {"workload": f"cfg3 {n_streams} streams/GPU x {n_total} samples, {n_win} windows of 48000 "
                                   f"per stream, all {n_win * n_streams} windows in one forward, then the sequential "
                                   f"PIT-L1 + append chain per window (PIT sums all-reduced over ranks)",
                       "global_batch": world * n_streams, "seq_len": 48000,
                       "parallelism": f"dp{world} (stream shards; 32-byte PIT all-reduce per window)"},
            "audio_seconds_per_second": round(windows / el * save_sec, 2),
        }
        emit(out)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: about half a second of sustained load, STEADY_STEPS)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps first (default: about 0.1 s, STEADY_STEPS: the GPU's clocks ramp under load)")
    ap.add_argument("--batch", type=int, default=None, help="utterances per GPU per step (default: the workload's)")
    ap.add_argument("--samples", type=int, default=None)
    ap.add_argument("--split", type=int, default=DEFAULT_SPLIT,
                    help="concurrent utterance chunks per forward (internal streams; bitwise-identical results)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--precision", default="f16x3", choices=["f16x3", "fp32", "bf16", "f16"],
                    help="GEMM arithmetic: f16x3 / fp32 meet the fp32 parity gates (default f16x3); bf16 / f16 are "
                         "the reduced-precision arms (BASELINE cfg 2 / cfg 5; tolerance in DESIGN.md §4)")
    ap.add_argument("--wlo", default="i8", choices=["f16", "e4m3", "i8"],
                    help="storage of the f16x3 weight lo plane in the fused TCN (include/sepvad.h SEPVAD_WLO_*): i8 "
                         "(default) / e4m3 (3 B per weight) or f16 (4 B)")
    ap.add_argument("--workload", default="offline", choices=["offline", "cfg4", "cfg5", "long", "stream"],
                    help="offline: cfg 2 (default, the BASELINE metric: B=64, N=32000); cfg4: 8 s reverberant "
                         "mixtures, B=64/GPU, N=64000 (T=251); cfg5: B=128/GPU, N=32000 (run with --precision "
                         "f16 for the fp16 arm); long: 16 s files as only_inference.py forwards them (B=8/GPU, "
                         "N=256000, T=1001: fused groups of 32 workgroups; --samples 480000 --batch 4 for 30 s files, groups of 59 "
                         "spanning XCDs); stream: cfg 3 streaming wrapper")
    args = ap.parse_args()
    steps, warmup = STEADY_STEPS[args.workload]
    args.steps = steps if args.steps is None else args.steps
    args.warmup = warmup if args.warmup is None else args.warmup
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    hold_stdout()
    if args.workload == "stream":
        return bench_stream(args)

    dist, world, rank, local_rank = init_dist(args)
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    cfg = pkg.CONFIG_WITH_VAD
    import contextlib
    # the constructor prints the merged config like the reference (model/model.py:371); keep stdout
    # to the single JSON line the driver parses
    with contextlib.redirect_stdout(sys.stderr):
        net = pkg.SeparationModel(**cfg)
    sd = synth.make_state_dict(cfg, 1234)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    net = net.eval().to(dev)
    net.native_precision = args.precision
    net.native_weight_lo = args.wlo
    B0, N0 = {"offline": (B_PER_GPU, N_SAMPLES), "cfg4": (64, 64000), "cfg5": (128, 32000),
              "long": (8, 256000)}[args.workload]
    B = args.batch or B0
    N = args.samples or N0
    T = 1 + N // 256
    # this rank's shard of utterances: global utterance ids [rank*B, (rank+1)*B)
    if args.workload == "cfg4":  # image-method reverberant mixtures (RT60 U[0.2, 0.6] s; host RIR generator)
        x, _ = synth.make_reverb_batch(B, N, 40_000 + rank * B)
    else:
        x, _ = synth.make_batch(B, N, 10_000 + rank * B)
    x = torch.from_numpy(x).to(dev)
    h = net.native_handle(dev)
    h.reserve(B, N)
    h.set_split(args.split)

    def step():
        with torch.no_grad():
            return net(x)

    # timed region (value)
    el = timed_region(step, args.steps, args.warmup, dist, torch.cuda.synchronize, _reduce_dev(dist, dev))

    # per-kernel timing pass (HIP events on the kernels' stream), same steps
    h.set_timing(True)
    gemm_ms = res_ms = tot_ms = 0.0
    n_res = n_gemm = 0
    for _ in range(max(3, min(args.steps, 10))):
        step()
        tm = h.timing()
        gemm_ms += tm["gemm_ms"]; res_ms += tm["res_out_ms"]; tot_ms += tm["total_ms"]
        n_res += tm["res_out_launches"]; n_gemm += tm["gemm_launches"]
    h.set_timing(False)
    fused = h.fused_status()  # synchronises; raises if a fused hand-off gave up
    # two-slice launches stream the int8 lo plane's values as fp16 (api.hip twfq, SEPVAD_TCN_WQ16): 4 bytes per weight
    wlo_streamed, nsl = args.wlo, (h.fused_slices() if fused else 1)
    if fused and args.precision == "f16x3" and args.wlo == "i8" and nsl == 2 \
            and os.environ.get("SEPVAD_TCN_WQ16", "1") != "0":
        wlo_streamed = "f16"

    if rank == 0:
        total_utt = world * B * args.steps
        value = total_utt / el
        res_avg_s = res_ms / n_res / 1e3
        if fused:
            # dominant kernel = the fused persistent TCN (all 24 blocks in one launch)
            flops_launch, bytes_launch = tcn_flops(B, T, args.precision), tcn_bytes(B, T, args.precision, wlo_streamed)
            body = ("k_tcn<LD_RECURSIVE> (fused persistent TCN: 24 x [conv1d 256->256, depthwise conv, res_out "
                    "512->256, TF-attention, recursive LN] + output head 256->514 and VAD conv1_1 taps, ")
            if args.precision == "f16x3":
                peak = F16_MFMA_PEAK_TFLOPS / 3.0
                kern = body + "fp16x3 split on v_mfma_f32_32x32x16_f16: peak = 2.5 PF/s / 3)"
            elif args.precision == "fp32":
                peak = FP32_MFMA_PEAK_TFLOPS
                kern = body + "exact fp32 on v_mfma_f32_32x32x2_f32, fp32 weights streamed: peak = 157.3 TF/s)"
            else:
                peak = F16_MFMA_PEAK_TFLOPS
                kern = body + f"{args.precision} operands on v_mfma_f32_32x32x16_{args.precision}: peak = 2.5 PF/s)"
            pmc_name = PMC_FILE_FUSED
        else:
            flops_launch, bytes_launch = res_out_flops(B, T), res_out_bytes(B, T)
            pmc_name = PMC_FILE
            # peak of the arithmetic actually issued: fp16x3 issues 3 fp16 MFMA products per fp32 product
            if args.precision == "f16x3":
                peak, kern = F16_MFMA_PEAK_TFLOPS / 3.0, ("k_gemm<F16X3,LD_SPLIT,EP_BIAS_ATT> (DepthConv1d.res_out "
                                                         "512->256; fp16x3 split on v_mfma_f32_32x32x16_f16: peak "
                                                         "= 2.5 PF/s / 3)")
            else:
                peak, kern = FP32_MFMA_PEAK_TFLOPS, ("k_gemm<F32,LD_PLAIN,EP_BIAS_ATT> (DepthConv1d.res_out 512->256, "
                                                     "v_mfma_f32_32x32x2_f32)")
        achieved = flops_launch / res_avg_s / 1e12
        fwd_timed = n_gemm / (1 if fused else 2 * 24 + 1)  # GEMM-bearing launches per forward
        all_gemm_tflops = gemm_flops_per_utt(T) * B * fwd_timed / (gemm_ms / 1e3) / 1e12 if gemm_ms > 0 else None
        # HBM bytes per launch of the same kernel from the committed rocprofv3 PMC passes
        # (tools/gpu_round.sh -> tools/pmc.py; FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md corrections)
        traffic = traffic_src = None
        pmc = os.path.join(REPO, "profiles", pmc_name)
        if (os.path.exists(pmc) and args.precision == "f16x3" and (not fused or args.wlo == PMC_WLO) and B == B_PER_GPU
                and N == N_SAMPLES):
            try:
                traffic = round(json.load(open(pmc))["hbm_bytes_per_launch"])
                traffic_src = "profiles/" + pmc_name
            except (OSError, ValueError, KeyError):
                traffic = None
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "utterances/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # arithmetic type of the path's GEMMs: the fp16x3 split (fp32-accurate by measurement, not IEEE fp32: the
            # weight lo plane keeps steps of 2^-19 of each row's largest weight), exact fp32
            # (v_mfma_f32_32x32x2_f32), or the reduced arm's operand; everything outside the GEMMs is fp32
            "dtype": {"f16x3": "f16x3 (fp32-accurate)", "fp32": "fp32", "bf16": "bf16", "f16": "f16"}[args.precision],
            "ieee_fp32": args.precision == "fp32",
            "gemm_arithmetic": args.precision + (f" (weight lo plane {args.wlo}"
                                                 + (", streamed as fp16" if wlo_streamed != args.wlo else "") + ")"
                                                 if args.precision == "f16x3" else ""),
            "split": args.split,
            "schedule": "fused" if fused else "multi-kernel",
            "data": "synthetic: seeded PCG64 2-speaker mixtures (0 dB SIR, noise SNR U[0,15] dB) and PCG64 "
                    "recipe weights (pretrained .pth absent from the reference)",
            "config": {
                "workload": {"offline": f"cfg2 config_with_vad.json forward, B={B}/GPU, N={N} samples (4 s @ 8 kHz "
                                        f"resampled to 16 kHz), T={T} frames",
                             "cfg4": f"cfg4 config_with_vad.json forward on image-method reverberant mixtures, "
                                     f"B={B}/GPU, N={N} samples (8 s @ 8 kHz), T={T} frames",
                             "cfg5": f"cfg5 config_with_vad.json forward, B={B}/GPU, N={N} samples, T={T} "
                                     f"frames, {args.precision} GEMMs",
                             "long": f"long files (only_inference.py:90-91 forwards a whole file), config_with_vad.json, "
                                     f"B={B}/GPU, N={N} samples ({N / 16000:.1f} s @ 16 kHz), T={T} frames"}[args.workload]
                            + "; full forward: STFT, 24 TCN blocks, VAD, iSTFT, est (side attributes on read)",
                "global_batch": world * B,
                "seq_len": N,
                "parallelism": f"dp{world} (independent utterance shards, no data-path collective)",
            },
            "roofline": {
                "bound": "mfma",
                "kernel": kern,
                "achieved": round(achieved, 3),
                "peak": round(peak, 1),
                "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": bytes_launch,
                "flops_per_launch": flops_launch,
                "avg_launch_us": round(res_avg_s * 1e6, 2),
                "all_gemms_tflops": round(all_gemm_tflops, 3) if all_gemm_tflops else None,
                "gemm_share_of_forward": round(gemm_ms / tot_ms, 3) if tot_ms > 0 else None,
            },
        }
        if fused:
            out["roofline"]["weight_stream"] = weight_stream(B, T, args.precision, res_avg_s, wlo=wlo_streamed, nsl=nsl)
            if args.precision == "f16x3" and args.wlo == PMC_WLO and B == B_PER_GPU and N == N_SAMPLES:
                out["roofline"]["caches"] = cache_counters(args.wlo)
            # the same fraction from the committed rocprofv3 average of the kernel (headline configuration only)
            if args.precision == "f16x3" and args.wlo == PMC_WLO and B == B_PER_GPU and N == N_SAMPLES:
                rp = rocprof_avg_us(TCN_KERNEL_PREFIX)
                if rp:
                    out["roofline"]["rocprof"] = {"avg_launch_us": round(rp, 2),
                                                  "achieved": round(flops_launch / (rp * 1e-6) / 1e12, 3),
                                                  "frac": round(flops_launch / (rp * 1e-6) / 1e12 / peak, 4),
                                                  "source": "profiles/" + STATS_FILE}
        if world == 1 and not args.no_cpu_baseline and args.workload == "offline":
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        emit(out)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
