"""Throughput benchmark of the MI355X split-CNN step (BASELINE.json metric: training samples/sec).

  python bench.py [--gpus N --steps K --warmup W --batch B --topology T]
  (N > 1: launched by torch.distributed.run, one process per GPU, RCCL over xGMI)

N = 1 (BASELINE config 2, "K2"): both stages fused on one MI355X, synthetic 1x28x28 batches of 4096,
fp32, the whole step (client fwd -> cut hand-off -> server fwd/CE/bwd/SGD -> client bwd/SGD)
replayed as one HIP graph. Inputs are resident in HBM before the timed region (a pool of batches,
copied into the graph's static input buffers inside each step).

N > 1: `value` is BASELINE's topology for that N: N = 2 -> config 3 ("K3", client GPU <-> server GPU,
micro-batched RCCL send/recv); N >= 3 -> config 4 ("K4", SplitFed: N-1 client GPUs feeding one server
GPU on the reference cut, client-gradient all-reduce). The RCCL p2p rate is measured first, the cut
exchange (dense fp32 or the lossless sparse codec) predicted from it and decided by a short trial of
both; "exchange" reports the choice and the cut-exchange GB/s per link and direction against the
measured p2p peak and the vendor link figure. Side objects: "replicated_dp" (data-parallel SplitFed-V1
replicas of the fused K2 step — NOT a BASELINE config) and "k5_splitfed" (config 5's widened model on
the hub topology). --topology replicated makes the replicas the headline instead.

One JSON line on rank 0 with the driver's contract plus "roofline" (dominant kernel, measured live
with HIP events on the launch stream in an eager pass after the timed region) and "cpu_baseline"
(rank 0, N = 1 only: the reference's client/server loop restated on torch CPU over FastAPI/HTTP +
pickle, B = 64, timed on this host — oracle/cpu_loop.py).
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

FLOP_PER_SAMPLE = 65_032_704          # total algorithmic FLOPs per training sample (direct conv)
CONV2_FLOP_PER_SAMPLE = 21_233_664    # each of conv2 fwd / dgrad / wgrad as a direct convolution
# conv2 runs as Winograd F(2x2,3x3) (csrc/slk_wino.hip): the MFMA work the algorithm needs per sample is
# 16 transform-domain GEMMs, 2 * 16 * M * N * K with (M, N, K) = fwd (64 co, 144 tiles, 32 ci),
# dgrad (32 ci, 169 tiles, 64 co), wgrad (64 co, 32 ci, 144 tiles). The roofline is priced on these.
WINO_FLOP_PER_SAMPLE = {"conv2_fwd_pool": 9_437_184, "conv2_dgrad": 11_075_584, "conv2_wgrad": 9_437_184}
STEP_FLOP_EXECUTED = FLOP_PER_SAMPLE - 3 * CONV2_FLOP_PER_SAMPLE + sum(WINO_FLOP_PER_SAMPLE.values())
FP32_PEAK_TFLOPS = 157.3              # MI355X_MICROARCH.md: fp32 matrix = vector peak
HBM_PEAK_GBS = 8000.0
CUT_BYTES = 86_528                    # fp32 [32,26,26] per sample, each direction
# widened split CNN (BASELINE config 5, splitcnn/wide.py): algorithmic FLOPs per training sample
WIDE_CONV_FLOP = {"wide_conv2_fwd": 150_994_944, "wide_conv3_fwd": 150_994_944, "wide_conv3_dgrad": 150_994_944,
                  "wide_conv2_dgrad": 150_994_944, "wide_conv3_wgrad": 150_994_944, "wide_conv2_wgrad": 150_994_944}
WIDE_FLOP_PER_SAMPLE = 914_030_592    # 6 x 150,994,944 (conv2/conv3) + 2 x 3,538,944 (conv1) + 3 x 327,680 (fc)
BF16_PEAK_TFLOPS = 2500.0             # MI355X_MICROARCH.md: dense bf16 MFMA peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096, help="per-GPU (per-client) batch")
    ap.add_argument("--topology", default="auto", choices=["auto", "replicated", "pipeline", "hub"])
    ap.add_argument("--micro", type=int, default=4, help="micro-batches of the pipeline / hub topologies")
    ap.add_argument("--no-micro-trial", action="store_true",
                    help="N > 1: time only --micro micro-batches in the exchange trial (default: also 2x --micro)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "dense", "codec"],
                    help="pipeline / hub cut exchange: auto = measure the link, then the faster of a short trial "
                         "of each; dense = fp32 cut + gradient; codec = the lossless sparse codec")
    ap.add_argument("--dense-exchange", action="store_true", help="= --exchange dense")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-pass", action="store_true")
    ap.add_argument("--no-exchange-phase", action="store_true")
    ap.add_argument("--exchange-steps", type=int, default=10, help="steps of the N > 1 side objects")
    ap.add_argument("--trial-steps", type=int, default=5,
                    help="timed steps per exchange trial at N > 1 (at least 5; the trial picks the lowest median)")
    ap.add_argument("--config", default="k2", choices=["k2", "k5"],
                    help="k2 = reference split CNN fp32 (headline); k5 = widened bf16 split CNN")
    ap.add_argument("--no-k5", action="store_true", help="skip the widened-config side measurement")
    ap.add_argument("--k5-batch", type=int, default=4096)
    ap.add_argument("--conv", default=None, choices=["x3", "x3w", "f32"],
                    help="K2 conv2 kernels: x3 = f16 MFMA with hi/lo-split fp32 operands for the forward, dgrad "
                         "and wgrad; x3w = x3 forward + dgrad with the Winograd f32 wgrad; f32 = Winograd "
                         "F(2x2,3x3) on the f32 MFMA throughout (default: splitcnn.engine.CONV_DEFAULT)")
    ap.add_argument("--no-conv-compare", action="store_true",
                    help="skip the short run of the other conv preset reported beside the headline")
    ap.add_argument("--no-images", action="store_true",
                    help="dense exchange of the f32 cut instead of the client's x3 split images (same bytes)")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the reference's step code on the drop-in modules (side object)")
    ap.add_argument("--no-hub-loopback", action="store_true",
                    help="skip the 1-GPU loopback of the K4 hub server's compute (7 clients x --micro chunks)")
    return ap.parse_args()


def cpu_baseline(seconds: float):
    """The reference loop on this host's CPU (child process; runs before this process touches
    the GPU)."""
    cmd = [sys.executable, "-m", "oracle.cpu_loop", "--seconds", str(seconds), "--batch", "64"]
    try:
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=seconds + 120)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
        d = json.loads(line)
    except Exception as e:  # reported, never fatal
        return {"value": None, "unit": "samples/s", "error": repr(e)[:300]}
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = "?"
    aff = d.get("affinity_cpus") or d.get("nproc")
    st, ct = d.get("server_threads"), d.get("client_threads")
    return {"value": round(d["value"], 1), "unit": "samples/s",
            # cores = the torch threads that actually compute: the client blocks on the server's reply and
            # the server on the client's request, so the two processes alternate and at most max(server,
            # client) threads run at once (torch's default thread count, i.e. OMP_NUM_THREADS where set)
            "cores": max(t for t in (st, ct) if t) if (st or ct) else aff,
            "kind": "port",
            "sample": f"{d['steps']} steps x B=64 in {d['seconds']:.1f}s: torch-CPU client+server processes "
                      f"over FastAPI/uvicorn + requests + pickle on localhost (src/client_part.py:103-138 <-> "
                      f"src/server_part.py:25-58, MLflow omitted) at torch's default thread count: server={st} "
                      f"client={ct} threads (OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}), "
                      f"which alternate; affinity mask {aff} CPUs, machine nproc={d.get('nproc')} ({model})"}


def make_pool(B, n, device, seed=42):
    import torch

    from splitcnn.data import SyntheticMNIST
    data = SyntheticMNIST(seed)
    xs, ys = zip(*(data.batch(B) for _ in range(n)))
    return torch.stack(xs).to(device), torch.stack(ys).to(device)


def timed(fn, K, W, device, group=None):
    """W warm-up calls, then K timed calls bracketed by barrier + synchronize; max over ranks."""
    import torch
    import torch.distributed as dist
    for i in range(W):
        fn(i)
    torch.cuda.synchronize(device)
    if dist.is_initialized():
        dist.barrier(group=group)
    t0 = time.perf_counter()
    for i in range(K):
        fn(W + i)
    torch.cuda.synchronize(device)
    if dist.is_initialized():
        dist.barrier(group=group)
    dt = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        dt = float(t.item())
    return dt


def kernel_pass(run_eager, K, device):
    """Eager steps with HIP events around each launch (on the launch stream)."""
    from splitcnn.engine import TIMER
    TIMER.reset()
    TIMER.enabled = True
    try:
        for i in range(K):
            run_eager(i)
        return TIMER.summary()
    finally:
        TIMER.enabled = False


def pmc_traffic(name, B):
    """HBM bytes per launch of kernel `name` at batch B from profiles/traffic.json (rocprofv3 --pmc
    FETCH_SIZE x2 + WRITE_SIZE, tools/pmc.sh + tools/pmc_summary.py), or None if not collected."""
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        return json.load(open(tpath)).get(name, {}).get(str(B))
    except (OSError, ValueError):
        return None


# Algorithmic HBM bytes per sample of each conv2 launch as the default fused step runs it (the minimum
# each must move: inputs read once, outputs written once):
#   fwd (x3i):  act16 images 86,528 read + pooled 36,864 + code 9,216 written
#   dgrad:      dpooled 36,864 + code 9,216 read (+ x 3,136 read when the client backward is fused into it,
#               + the cut gradient 86,528 written when it is not)
#   wgrad (x3s): act16 86,528 + dpooled 36,864 + code 9,216 read
ALGO_BYTES = {"conv2_fwd_pool": 132_608, "conv2_dgrad": 46_080, "conv2_wgrad": 132_608}
# kernel symbols in rocprofv3's --stats summary, per (TIMER name, variant)
ROCPROF_SYMBOL = {("conv2_dgrad", "x3_fused"): "conv2_dgrad_x3_kernel<true>",
                  ("conv2_dgrad", "x3"): "conv2_dgrad_x3_kernel<false>",
                  ("conv2_fwd_pool", "x3_images"): "conv2_fwd_pool_x3_kernel<true>",
                  ("conv2_wgrad", "x3_images"): "conv2_wgrad_x3p_kernel"}


def rocprof_avg(symbol, pattern="kernel_stats_k2.csv"):
    """Average duration (ms) of `symbol` in the committed rocprofv3 --stats summary of the same bench
    command, profiles/rocprof_<pattern>, with the slk_build_id of the library it profiled (the
    `.build_id` file written next to it by tools/gpu_profile_all.sh). Returns (ms, source, build id,
    whether that id is the loaded library's) or Nones."""
    import csv
    f = os.path.join(ROOT, "profiles", "rocprof_" + pattern)
    try:
        bid = open(os.path.splitext(f)[0] + ".build_id").read().strip()
    except OSError:
        bid = None
    try:
        from splitcnn import _lib
        current = _lib.build_id()
    except Exception:  # noqa: BLE001
        current = None
    try:
        for row in csv.DictReader(open(f)):
            if symbol in row["Name"]:
                return (round(float(row["AverageNs"]) / 1e6, 4), os.path.relpath(f, ROOT), bid,
                        bid is not None and bid == current)
    except (OSError, KeyError, ValueError):
        pass
    return None, None, None, False


def conv_roofline(name, avg_ms, B, impl):
    """Roofline of one conv2 launch. wino: its transform-domain GEMM FLOPs on the f32 MFMA peak; x3: the
    f16 MFMA FLOPs it executes (3 products per direct-conv multiply-add) on the dense f16 peak."""
    direct_eq = CONV2_FLOP_PER_SAMPLE * B / (avg_ms * 1e-3) / 1e12
    if impl == "x3":
        flops, peak = 3 * CONV2_FLOP_PER_SAMPLE * B, BF16_PEAK_TFLOPS
        algo = ("direct implicit GEMM on v_mfma_f32_16x16x32_f16, f32 operands split hi/lo (3 MFMAs per "
                "product, f32 accumulate; flop_per_launch = the f16 MFMA FLOPs executed)")
    else:
        flops, peak = WINO_FLOP_PER_SAMPLE[name] * B, FP32_PEAK_TFLOPS
        algo = "Winograd F(2x2,3x3), f32 MFMA (flop_per_launch = its transform-domain GEMMs)"
    ach = flops / (avg_ms * 1e-3) / 1e12
    r = {"kernel": name, "bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
         "frac": round(ach / peak, 4), "traffic": pmc_traffic(name + ("_x3" if impl == "x3" else ""), B),
         "flop_per_launch": flops, "avg_ms": round(avg_ms, 4), "algorithm": algo,
         "direct_conv_equivalent_tflops": round(direct_eq, 2)}
    if impl == "x3" and name == "conv2_wgrad" and wgrad_x3_form() == 2:
        # round 6: the 2:4-sparse f16 MFMA issues half of those products (the routed dY's structural zeros are
        # skipped); priced against the SPARSE peak (2x the dense one) the kernel's executed work sits at:
        r["algorithm"] = ("direct implicit GEMM on v_smfmac_f32_16x16x64_f16 (2:4 sparse: dY has <= 2 nonzeros in "
                          "every 4-pixel block of a row), f32 operands split hi/lo (3 products); flop_per_launch = "
                          "the dense-equivalent f16 FLOPs (structural zeros included), half of them issued")
        r["frac_of_sparse_peak"] = round(ach / (2 * peak), 4)
    return r


def _query_or_none(name):
    try:
        from splitcnn import _lib
        return _lib.query(name)
    except Exception:  # noqa: BLE001
        return None


def wgrad_x3_form():
    """slk_conv2_wgrad_x3_form() of the loaded library (2 = sparse MFMA, 1 = dense x3), None without one."""
    try:
        from splitcnn import _lib
        return _lib.query("slk_conv2_wgrad_x3_form")
    except Exception:  # noqa: BLE001
        return None


def roofline_from(kern, B, impls=None, variants=None):
    conv = {k: v for k, v in kern.items() if k.startswith("conv2_")}
    if not conv:
        return None
    impls = impls or {}
    name = max(conv, key=lambda k: conv[k]["avg_ms"])
    r = conv_roofline(name, conv[name]["avg_ms"], B, impls.get(name, "wino"))
    variant = (variants or {}).get(name)
    if variant is not None:
        algo = ALGO_BYTES[name] * B
        if name == "conv2_dgrad":
            algo += (3_136 if variant == "x3_fused" else 86_528) * B
        r["traffic_algorithmic"] = algo
        r["traffic_ratio"] = round(r["traffic"] / algo, 3) if r.get("traffic") else None
        sym = ROCPROF_SYMBOL.get((name, variant))
        if sym:
            ms, src, bid, same = rocprof_avg(sym)
            # only a profile of THIS library build counts as the cross-check; an older one is labelled
            r["rocprof_avg_ms" if same else "rocprof_avg_ms_historical"] = ms
            r["rocprof_source"] = src
            r["rocprof_build_id"] = bid[:16] if bid else None
            r["hip_event_avg_ms"] = r["avg_ms"]
            if same and ms:
                # the same launch priced on the profiler's duration, next to `frac` (this process's events)
                r["frac_rocprof"] = round(r["flop_per_launch"] / (ms * 1e-3) / 1e12 / r["peak"], 4)
                # the profiled process's own JSON line (written beside the summary by tools/gpu_profile_all.sh):
                # its step time and its own HIP-event average of this kernel, so the two clocks are comparable
                try:
                    pj = json.load(open(os.path.join(ROOT, "profiles", "rocprof_kernel_stats_k2.bench.json")))
                    r["rocprof_process"] = {"ms_per_step": round(pj["ms_per_step"], 4),
                                            "graph": pj.get("config", {}).get("graph"),
                                            "hip_event_avg_ms": (pj.get("roofline") or {}).get("avg_ms")}
                except (OSError, ValueError, KeyError, TypeError):
                    pass
    r["per_kernel"] = {k: {kk: vv for kk, vv in conv_roofline(k, v["avg_ms"], B, impls.get(k, "wino")).items()
                           if kk in ("avg_ms", "achieved", "peak", "frac", "direct_conv_equivalent_tflops",
                                     "frac_of_sparse_peak")}
                       for k, v in conv.items()}
    return r


def run_single(args, out):
    import torch

    from splitcnn.data import init_models
    from splitcnn.engine import SplitTrainer
    dev = torch.device("cuda:0")
    B = args.batch
    X, Y = make_pool(B, 4, dev)
    from splitcnn.engine import CONV_DEFAULT, CONV_PRESETS
    conv = args.conv or CONV_DEFAULT
    a, b = init_models(seed=0)
    tr = SplitTrainer(a, b, device=dev, graph=not args.no_graph, conv=conv)
    for i in range(4):   # the pool is the loader's ring: one graph per buffer pair, captured before timing
        tr.register_inputs(X[i], Y[i])
    step = lambda i: tr.step(X[i % 4], Y[i % 4])  # noqa: E731
    dt = timed(step, args.steps, args.warmup, dev)
    losses = tr.loss_log.flush()
    out.update(value=args.steps * B / dt, ms_per_step=dt / args.steps * 1e3)
    fi, di, wi = CONV_PRESETS[conv]
    out["config"] = {"workload": "K2: split CNN (model_def.py ModelPartA+ModelPartB) both stages fused on "
                                 "1xMI355X, synthetic 1x28x28 MNIST-shape batches, fp32, HIP-graph step",
                     "global_batch": B, "per_gpu_batch": B, "topology": "fused-1gpu",
                     "graph": not args.no_graph, "conv": conv,
                     "conv2_kernels": {"fwd_pool": fi, "dgrad": di, "wgrad": wi},
                     "cut_handoff": ("client conv1 writes the x3 split input images (slk_conv1_fwd_x3); no f32 cut"
                                     if tr.client.emit_act16 else "f32 cut"),
                     "client_backward": ("fused into the x3 dgrad (slk_conv2_dgrad_x3_c1w); no cut gradient in HBM"
                                         if tr.fuse_client_backward else "cut gradient -> conv1 wgrad"),
                     "arithmetic": "fp32 tensors, f32 accumulation; conv2 'x3' kernels multiply f32 operands split "
                                   "into f16 hi + lo (3 MFMA products, per-product error <= ~7e-7 relative, "
                                   "checked vs fp64 at the f32 path's bars), 'wino' = Winograd on the f32 MFMA"}
    out["loss_first_last"] = [round(losses[0][1], 5), round(losses[-1][1], 5)] if losses else None
    if not args.no_kernel_pass:
        # (before the preset comparison: the headline's roofline must not depend on the other presets)
        try:
            tr2 = SplitTrainer(*init_models(seed=0), device=dev, graph=False, conv=conv)
            kern = kernel_pass(lambda i: tr2.step(X[i % 4], Y[i % 4]), max(3, min(args.steps, 10)), dev)
            out["kernels"] = {k: round(v["avg_ms"], 4) for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["avg_ms"])}
            variants = {"conv2_dgrad": ("x3_fused" if tr2.fuse_client_backward else di),
                        "conv2_fwd_pool": ("x3_images" if tr2.client.emit_act16 else fi),
                        "conv2_wgrad": ("x3_images" if tr2.client.emit_act16 else wi)}
            out["roofline"] = roofline_from(kern, B, {"conv2_fwd_pool": fi, "conv2_dgrad": di, "conv2_wgrad": wi},
                                            variants)
            try:  # this box's sustained f16 MFMA rate: the pool's boxes differ by several per cent under load
                from splitcnn import ops
                box = ops.mfma_probe_tflops(dev)
                r = out["roofline"]
                r["box_probe"] = {"mfma_f16_dense_tflops": round(box, 1), "nominal_tflops": BF16_PEAK_TFLOPS,
                                  "ratio": round(box / BF16_PEAK_TFLOPS, 4),
                                  "probe": "slk_mfma_probe: 6 independent v_mfma_f32_16x16x32_f16 chains per wave, "
                                           "2 waves per SIMD, varied operands; median of 3 launches"}
                if r.get("unit") == "TFLOP/s" and r.get("achieved"):
                    r["frac_of_box_probe"] = round(r["achieved"] / box, 4)
            except Exception as e:  # reported, never fatal
                out["roofline"]["box_probe"] = {"error": repr(e)[:200]}
            if tr2.fuse_client_backward and out["roofline"].get("kernel") == "conv2_dgrad":
                out["roofline"]["note"] = ("conv2_dgrad here also runs the client's ReLU backward + conv1 wgrad in "
                                           "its epilogue (slk_conv2_dgrad_x3_c1w); those FLOPs are not counted, its "
                                           "time is; traffic = the fused launch's PMC bytes (profiles/traffic.json), "
                                           "traffic_algorithmic = dpooled + code + x read once")
            del tr2
        except Exception as e:  # the headline stands on its own
            out["roofline"] = {"error": repr(e)[:300]}
    if not args.no_conv_compare:
        out["conv_presets"] = {conv: round(out["value"], 1)}
        for other in CONV_PRESETS:
            if other == conv:
                continue
            try:
                tro = SplitTrainer(*init_models(seed=0), device=dev, graph=not args.no_graph, conv=other)
                for i in range(4):
                    tro.register_inputs(X[i], Y[i])
                dto = timed(lambda i: tro.step(X[i % 4], Y[i % 4]), args.steps, args.warmup, dev)
                out["conv_presets"][other] = round(args.steps * B / dto, 1)
                del tro
            except Exception as e:  # reported, never fatal to the headline
                out["conv_presets"][other] = {"error": repr(e)[:300]}
    if conv == "f32":  # every conv2 FLOP on the f32 MFMA: one peak prices the whole step
        out["step_roofline_frac"] = round(out["value"] * STEP_FLOP_EXECUTED / (FP32_PEAK_TFLOPS * 1e12), 4)
    out["step_direct_equivalent_tflops"] = round(out["value"] * FLOP_PER_SAMPLE / 1e12, 2)


def run_dropin(X, Y, steps, warmup):
    """The reference's own step code (src/client_part.py:112-133 <-> src/server_part.py:45-57, HTTP and
    pickle removed) on the drop-in modules (splitcnn.model_def: torch.library ops over the x3 kernels,
    library.py) at the K2 batch: eager autograd + torch.optim.SGD, the payload clone, the server's
    .grad clone and the per-step loss.item() of its log_metric call (server_part.py:55)."""
    import torch

    from splitcnn.data import init_models
    from splitcnn.library import conv_impls
    from splitcnn.model_def import CrossEntropyLoss
    dev = X.device
    client, server = (m.to(dev) for m in init_models(seed=0))
    copt = torch.optim.SGD(client.parameters(), lr=0.01)
    sopt = torch.optim.SGD(server.parameters(), lr=0.01)
    criterion = CrossEntropyLoss()
    losses = []

    def step(i):
        data, target = X[i % 4], Y[i % 4]
        copt.zero_grad()
        activations = client(data)
        client_activations = activations.clone().detach()       # the payload (client_part.py:118)
        client_activations.requires_grad_(True)                  # server_part.py:45
        sopt.zero_grad()
        loss = criterion(server(client_activations), target)
        loss.backward()
        sopt.step()
        losses.append(loss.item())                               # mlflow.log_metric (server_part.py:55)
        cut_layer_gradient = client_activations.grad.clone().detach()
        activations.backward(cut_layer_gradient)                 # client_part.py:132-133
        copt.step()
    dt = timed(step, steps, warmup, dev)
    B = X.shape[1]
    return {"workload": "the reference's step code (client_part.py:112-133 / server_part.py:45-57, no HTTP) on "
                        "the drop-in ModelPartA/ModelPartB/CrossEntropyLoss modules, eager autograd + "
                        "torch.optim.SGD, loss.item() per step", "conv2_kernels": dict(zip(("fwd_pool", "dgrad", "wgrad"),
                                                                                          conv_impls())),
            "samples_per_s": round(steps * B / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3), "batch": B,
            "loss_first_last": [round(losses[0], 5), round(losses[-1], 5)]}


def run_hub_loopback(args, nc=7):
    """K4's bottleneck measured on ONE GPU: the hub server's step for nc clients x B samples (the chunked,
    graph-captured sequence dist.Hub.server_step runs: per micro-batch chunk of nc*B/m samples codec
    unpack -> forward / loss / backward -> codec pack; then one SGD step), with the chunks' inputs already
    in the server's receive buffers (no transport). Compared with the fused 1-GPU step minus the client's
    conv1 (which a hub server does not run), the server's rate bounds BASELINE config 4's throughput."""
    import torch

    from splitcnn import dist as sd
    from splitcnn.codec import CutCodec
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage, ServerStage
    dev = torch.device("cuda:0")
    B, m = args.batch, args.micro
    b, G = B // m, nc * B
    a, srv = init_models(seed=0)
    images = bool(args.dense_exchange) and not getattr(args, "no_images", False)
    hub = sd.Hub(ServerStage(srv, device=dev), rank=nc, world=nc + 1, micro=m, compress=not args.dense_exchange,
                 graph=not args.no_graph, images=images)
    codec = hub._use_codec(dev)
    hub._prepare(B, dev, codec)  # the chunk graphs (their warm-up zeroes the receive buffers)
    cl = ClientStage(a, device=dev)
    cl.emit_amax = True
    n = b * 32 * 26 * 26
    acts = hub._inputs(G, dev, codec)
    labels = hub._buf("labels", (G,), torch.int64, dev)
    amx = hub._buf("amax", (G,), torch.float32, dev)
    hub._buf("cuts", (G, 32, 26, 26), torch.float32, dev)
    hub._buf("loss_parts", (m,), torch.float32, dev)
    data = SyntheticMNIST(7)
    for k in range(m):
        for ci in range(nc):
            sl = slice(k * nc * b + ci * b, k * nc * b + (ci + 1) * b)
            x, y = data.batch(b)
            if images:
                cl.forward_images(x.to(dev), acts[sl.start * sd.IMG_BYTES:sl.stop * sd.IMG_BYTES], amx[sl])
            elif codec is not None:   # the client's f32 cut, encoded into the server's receive buffers
                ca = cl.forward(x.to(dev))
                amx[sl].copy_(cl._act_amax)
                codec.encode(ca, codec.buffers(("s", ci, k), n, dev))
            else:
                cl.forward(x.to(dev), out=acts[sl])
                amx[sl].copy_(cl._act_amax)
            labels[sl].copy_(y.to(dev))
    return hub, cl, codec, data, nc


def hub_loopback_rate(args, ref_value, conv1_ms):
    import torch
    hub, cl, codec, data, nc = run_hub_loopback(args)
    dev = torch.device("cuda:0")
    B, m = args.batch, args.micro
    b = B // m
    s = hub.stage
    parts = hub._bufs["loss_parts"]

    def step(i):
        for k in range(m):
            hub._run_chunk(k, B, dev, codec)
        s.step()
        s.log_loss(parts, scale=1.0)
    K = max(3, min(args.steps, 10))
    dt = timed(step, K, 2, dev)
    rate = K * nc * B / dt
    fused_minus_conv1 = B / (B / ref_value - conv1_ms * 1e-3) if ref_value and conv1_ms else None
    fused = hub._fused(codec)
    return {"workload": f"K4 hub server compute, {nc} clients x {B} samples in {m} chunks of {nc * b} "
                        f"(codec unpack/pack {'on' if codec is not None else 'off'}"
                        f"{' (fused: unpack into the x3 images, pack in the dgrad epilogue)' if fused else ''}"
                        f"{', x3 split images in' if hub.images else ''}, HIP graph per chunk), "
                        "inputs already in the receive buffers: the 1-GPU bound of BASELINE config 4",
            "samples_per_s": round(rate, 1), "ms_per_step": round(dt / K * 1e3, 3), "global_batch": nc * B,
            "fused_1gpu_minus_conv1_samples_per_s": round(fused_minus_conv1, 1) if fused_minus_conv1 else None,
            "ratio": round(rate / fused_minus_conv1, 3) if fused_minus_conv1 else None}


def run_wide(args, B, steps, warmup, kernel_pass_on=True):
    """BASELINE config 5: widened split CNN (bf16 MFMA convs, dropout, Adam) fused on one GPU."""
    import torch

    from splitcnn.wide import SyntheticCIFAR, WideTrainer, init_wide_models
    dev = torch.device("cuda:0")
    data = SyntheticCIFAR(42)
    xs, ys = zip(*(data.batch(B) for _ in range(4)))
    X, Y = torch.stack(xs).to(dev), torch.stack(ys).to(dev)
    tr = WideTrainer(*init_wide_models(seed=0), device=dev, graph=not args.no_graph)
    for i in range(4):
        tr.register_inputs(X[i], Y[i])
    dt = timed(lambda i: tr.step(X[i % 4], Y[i % 4]), steps, warmup, dev)
    losses = tr.loss_log.flush()
    r = {"metric": "training samples/sec, widened split CNN (BASELINE config 5)", "value": steps * B / dt,
         "unit": "samples/s", "ms_per_step": dt / steps * 1e3, "dtype": "bf16",
         "config": {"workload": "K5: widened split CNN (conv 3-64-128-256, 3x32x32, cut [256,8,8] after conv3; "
                                "server dropout + fc 16384->10; Adam), fused on 1xMI355X, bf16 MFMA "
                                "implicit-GEMM convs, HIP-graph step", "global_batch": B},
         "loss_first_last": [round(losses[0][1], 5), round(losses[-1][1], 5)] if losses else None,
         "step_roofline_frac": round(steps * B / dt * WIDE_FLOP_PER_SAMPLE / (BF16_PEAK_TFLOPS * 1e12), 4)}
    if kernel_pass_on:
        tr2 = WideTrainer(*init_wide_models(seed=0), device=dev, graph=False)
        kern = kernel_pass(lambda i: tr2.step(X[i % 4], Y[i % 4]), 3, dev)
        r["kernels"] = {k: round(v["avg_ms"], 4) for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["avg_ms"])}
        conv = {k: v for k, v in kern.items() if k in WIDE_CONV_FLOP}
        name = max(conv, key=lambda k: conv[k]["avg_ms"])
        ach = WIDE_CONV_FLOP[name] * B / (conv[name]["avg_ms"] * 1e-3) / 1e12
        r["roofline"] = {"kernel": name, "bound": "mfma", "achieved": round(ach, 1), "peak": BF16_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(ach / BF16_PEAK_TFLOPS, 4), "traffic": pmc_traffic(name, B),
                         "flop_per_launch": WIDE_CONV_FLOP[name] * B, "avg_ms": round(conv[name]["avg_ms"], 4)}
        # every conv kernel on its direct-convolution FLOPs; the weight gradients on the 2:4-sparse MFMA (round 6)
        # execute half the products as sparse instructions: also priced against the sparse peak (2x dense)
        sparse_wg = _query_or_none("slk_wide_wgrad_form") == 1
        per = {}
        for k, v in sorted(conv.items(), key=lambda kv: -kv[1]["avg_ms"]):
            a_k = WIDE_CONV_FLOP[k] * B / (v["avg_ms"] * 1e-3) / 1e12
            per[k] = {"achieved": round(a_k, 1), "frac": round(a_k / BF16_PEAK_TFLOPS, 4), "avg_ms": round(v["avg_ms"], 4)}
            if sparse_wg and k.endswith("_wgrad") and k != "wide_conv1_wgrad":
                per[k]["frac_of_sparse_peak"] = round(a_k / (2 * BF16_PEAK_TFLOPS), 4)
                per[k]["algorithm"] = "v_smfmac_f32_16x16x64_bf16 on the max-pool-routed dC (2 of every 4 pixels)"
        r["roofline"]["per_kernel"] = per
        r["conv_tflops"] = {k: round(WIDE_CONV_FLOP[k] * B / (v["avg_ms"] * 1e-3) / 1e12, 1) for k, v in conv.items()}
    return r


XGMI_LINK_GBPS = 153.6   # vendor per-link xGMI figure (task brief: 7 links x ~153 GB/s per GPU); convention unstated
# Server-side rates of the hub step on one GPU (bench k4_server_loopback; samples/s at B = 4096 per
# client): with the dense exchange the server runs the plain stage kernels, with the codec it also unpacks
# and packs. Used only for the exchange PREDICTION reported next to the measured trial that decides.
HUB_SERVER_RATE = {"dense": 5.1e6, "codec": 4.1e6}   # round 5: dense = the image exchange; codec = the fused server kernels
CODEC_WIRE_FRACTION = 0.456   # wire bytes / dense bytes of the codec on the synthetic data


def predict_exchange(nc, B, p2p_gbps):
    """Predicted step time of the hub per exchange: max(server compute of nc*B samples, one client link's
    cut bytes in one direction at the measured p2p rate) — the micro-batches overlap the two. Dense wins
    once the link sustains about 354 MB / (7 x 4096 / 4.4 M/s) = 55 GB/s per direction at nc = 7."""
    out = {}
    for ex, frac in (("dense", 1.0), ("codec", CODEC_WIRE_FRACTION)):
        server = nc * B / HUB_SERVER_RATE[ex]
        link = frac * B * CUT_BYTES / (p2p_gbps * 1e9) if p2p_gbps else float("inf")
        out[ex] = round(max(server, link) * 1e3, 3)
    return out


def timed_steps(fn, K, W, device, group=None):
    """W warm-up calls, then K calls each timed on its own between a synchronize + barrier; returns the K
    per-step times (s), each the max over ranks (one all-reduce at the end). The exchange trials choose
    by the median of these."""
    import torch
    import torch.distributed as dist
    for i in range(W):
        fn(i)
    ts = []
    for i in range(K):
        torch.cuda.synchronize(device)
        if dist.is_initialized():
            dist.barrier(group=group)
        t0 = time.perf_counter()
        fn(W + i)
        torch.cuda.synchronize(device)
        ts.append(time.perf_counter() - t0)
    if dist.is_initialized():
        t = torch.tensor(ts, dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        ts = [float(v) for v in t.cpu()]
    return ts


# executed f16 MFMA FLOPs per sample of the server GPU's three x3 conv2 kernels (forward, dgrad, wgrad; each
# does 3 f16 products per direct-conv multiply-add): what the server GPU's step-level roofline prices
SERVER_X3_FLOP_PER_SAMPLE = 9 * CONV2_FLOP_PER_SAMPLE


def server_kernel_pass(t, B, dev, steps=3):
    """Hub / Pipeline server rank, after the headline: `steps` eager passes over the step's chunks on the
    data already in the receive buffers (no exchange), HIP events around each launch on the launch
    stream; the dominant conv2 kernel priced per launch (one launch = one chunk of nc*B/m samples)."""
    from splitcnn.engine import TIMER
    codec = t._use_codec(dev)
    TIMER.reset()
    TIMER.enabled = True
    try:
        for _ in range(steps):
            for k in range(t.micro):
                t._chunk(k, B, dev, codec)
        kern = TIMER.summary()
    finally:
        TIMER.enabled = False
    s = t.stage
    CH = t.nclients * B // t.micro
    r = roofline_from(kern, CH, {"conv2_fwd_pool": s.impl_fwd, "conv2_dgrad": s.impl_dgrad, "conv2_wgrad": s.impl_wgrad})
    if r is not None:
        r["launch_batch"] = CH
        r["measured_on"] = "server rank, eager chunk passes after the timed region (HIP events on the launch stream)"
        r["kernels_ms"] = {k: round(v["avg_ms"], 4) for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["avg_ms"])}
    return r


def step_roofline(samples_per_s_per_server, ms_per_step, global_batch):
    """Step-level roofline of the server GPU at N > 1: the executed f16 MFMA FLOPs of its x3 conv2 kernels
    over the step time, against the dense f16 peak."""
    ach = samples_per_s_per_server * SERVER_X3_FLOP_PER_SAMPLE / 1e12
    return {"scope": "server GPU over the whole step (x3 conv2 forward + dgrad + wgrad: 9 x 21,233,664 executed "
                     "f16 MFMA FLOP per sample)", "bound": "mfma", "achieved": round(ach, 2), "peak": BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(ach / BF16_PEAK_TFLOPS, 4), "traffic": None,
            "flop_per_step": SERVER_X3_FLOP_PER_SAMPLE * global_batch, "ms_per_step": round(ms_per_step, 4),
            "step_direct_equivalent_tflops": round(samples_per_s_per_server * FLOP_PER_SAMPLE / 1e12, 2)}


# watchdog limits (s) per phase of the N > 1 bench; SLK_BENCH_WATCHDOG_SCALE multiplies them
PHASE_LIMIT_S = {"setup": 300, "p2p": 120, "trial": 150, "roofline": 120, "replicated": 240, "k5": 300, "teardown": 120}


def run_distributed(args, out, rank, world, local, wd=None):
    """N > 1, BASELINE's own topologies. Headline `value`: N = 2 -> K3 (client GPU <-> server GPU,
    micro-batched RCCL send/recv, dist.Pipeline); N >= 3 -> K4 (SplitFed: N-1 client GPUs feeding 1
    server GPU, client all-reduce, dist.Hub). Before timing: the RCCL p2p rate client 0 -> server is
    measured, the exchange (dense fp32 or the lossless sparse codec) is predicted from it, and a trial of
    both on the real topology decides (median of >= 5 timed steps). `roofline`: the server GPU's
    executed f16 FLOPs per step over the step time, with its dominant kernel (HIP events on the server
    rank) and the link beside it. Side objects: "replicated_dp" (data-parallel SplitFed-V1 replicas of the
    fused K2 step — NOT a BASELINE config) and "k5_splitfed" (config 5's widened model on the hub
    topology), with cut-exchange GB/s against the measured p2p peak and the vendor link figure. Every
    phase runs under the watchdog `wd`; every HIP graph of a phase is captured after a synchronize +
    barrier and before that phase's first exchange (capture mode thread_local besides)."""
    import torch
    import torch.distributed as dist

    from splitcnn import dist as sd
    from splitcnn.data import init_models
    from splitcnn.engine import ClientStage, ServerStage
    wd = wd or Watchdog(out, rank, enabled=False)
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    B = args.batch
    topo = args.topology if args.topology != "auto" else ("pipeline" if world == 2 else "hub")
    wd.phase("setup", PHASE_LIMIT_S["setup"])
    X, Y = make_pool(B, 4, dev, seed=42 + rank)
    grp = sd.client_group_for(world)   # every rank creates it (collective), used by hub topologies
    groups = sd.exchange_groups()      # one process group per exchange direction (see its docstring)
    nc = world - 1

    def settle():
        torch.cuda.synchronize(dev)
        dist.barrier()

    def build(topology, micro, codec):
        """Construct this rank's side of `topology`, then capture its graphs between two settle()s."""
        a, b = init_models(seed=0)
        images = not codec and not args.no_images
        if topology == "replicated":
            t = sd.Replicated(ClientStage(a, device=dev), ServerStage(b, device=dev), graph=not args.no_graph)
            fn, gb = (lambda i: t.step(X[i % 4], Y[i % 4])), world * B
        elif topology == "pipeline":
            assert world == 2
            if rank == 0:
                t = sd.Pipeline(ClientStage(a, device=dev), "client", 1, micro=micro, compress=codec, groups=groups,
                                graph=not args.no_graph, images=images)
                fn = lambda i: t.client_step(X[i % 4], Y[i % 4])  # noqa: E731
            else:
                t = sd.Pipeline(ServerStage(b, device=dev), "server", 0, micro=micro, compress=codec, groups=groups,
                                graph=not args.no_graph, images=images)
                fn = lambda i: t.server_step(B, dev)  # noqa: E731
            gb = B
        elif topology == "hub":
            if rank < world - 1:
                t = sd.Hub(ClientStage(a, device=dev), rank, world, client_group=grp, micro=micro, compress=codec,
                           groups=groups, graph=not args.no_graph, images=images)
                fn = lambda i: t.client_step(X[i % 4], Y[i % 4])  # noqa: E731
            else:
                t = sd.Hub(ServerStage(b, device=dev), rank, world, client_group=grp, micro=micro, compress=codec,
                           groups=groups, graph=not args.no_graph, images=images)
                fn = lambda i: t.server_step(B, dev)  # noqa: E731
            gb = (world - 1) * B
        else:
            raise ValueError(topology)
        settle()
        if topology == "replicated":
            t.prepare(B)
        else:
            t.prepare(B, dev)
        settle()
        return fn, t, gb

    labels = {
        "replicated": "data-parallel SplitFed-V1 replicas (NOT a BASELINE config): every GPU hosts one client + "
                      "one server replica of the reference split CNN, cut in place, one 444 KB gradient "
                      "all-reduce per step (= the reference step at the concatenated N*B batch)",
        "pipeline": "K3: 2xMI355X client-stage GPU <-> server-stage GPU, micro-batched RCCL send/recv of "
                    "activations and cut gradients (BASELINE config 3)",
        "hub": f"K4: SplitFed, {nc} client GPU(s) feeding 1 server GPU (reference cut), micro-batched RCCL "
               "send/recv, client-gradient all-reduce (BASELINE config 4)"}
    codec_label = {True: "lossless sparse codec: ReLU-cut bit mask + nonzero values out, gradient at those positions "
                         "back (bit-identical results)",
                   False: "dense: the client's x3 split images (f16 hi/lo, per-sample scale; the f32 cut's bytes) "
                          "+ per-sample max out, fp32 cut gradient back" if not args.no_images else "dense fp32"}

    def wire(t):
        """rank 0 is a client in both exchange topologies: its link's bytes (both directions, labels and
        codec headers included) actually moved vs what the dense exchange moves."""
        v = torch.tensor([float(getattr(t, "exchange_bytes", 0)), float(getattr(t, "dense_bytes", 0))],
                         dtype=torch.float64, device=dev)
        dist.broadcast(v, 0)
        return int(v[0].item()), int(v[1].item())

    # 1. the link: RCCL p2p client 0 -> server, one direction, one cut's worth of bytes
    peak = None
    wd.phase("p2p peak", PHASE_LIMIT_S["p2p"])
    try:
        p = sd.measure_p2p(CUT_BYTES * B, 0, world - 1, dev)
        pk = torch.tensor([p or 0.0], dtype=torch.float64, device=dev)
        dist.all_reduce(pk, op=dist.ReduceOp.MAX)
        peak = float(pk.item())
        out["p2p_peak_GBps_measured"] = round(peak, 2)
    except Exception as e:
        out["p2p_peak_GBps_measured"] = {"error": repr(e)[:300]}

    # 2. the exchange: predicted from the link, decided by a trial of both on this topology
    exch = {"vendor_link_GBps": XGMI_LINK_GBPS}
    if topo == "replicated":
        wd.phase("replicated: build + capture", PHASE_LIMIT_S["trial"])
        fn, t, global_batch = build(topo, args.micro, False)
    else:
        forced = {"dense": False, "codec": True}.get("dense" if args.dense_exchange else args.exchange)
        exch["prediction_ms_per_step"] = predict_exchange(nc if topo == "hub" else 1, B, peak)
        trials, spread = {}, {}
        built = {}
        # micro-batch counts tried: a link-bound pipeline takes ~(1 + 1/m) x its link time, while each
        # micro-batch adds fixed costs (p2p op latency, the codec's count round trip), so the link decides
        micros = [args.micro] + ([2 * args.micro] if not args.no_micro_trial and B % (2 * args.micro) == 0 else [])
        Kt = max(5, args.trial_steps)
        for name, codec in (("dense", False), ("codec", True)):
            if forced is not None and codec != forced:
                continue
            for m in micros:
                key = f"{name}/m{m}"
                wd.phase(f"{topo} x{world}: {key} exchange trial", PHASE_LIMIT_S["trial"])
                f, tt, gb = build(topo, m, codec)
                ts = timed_steps(f, Kt, 2, dev)
                trials[key] = round(statistics.median(ts) * 1e3, 3)
                spread[key] = [round(min(ts) * 1e3, 3), round(max(ts) * 1e3, 3)]
                built[key] = (f, tt, gb, m)
        best = min(trials, key=trials.get)
        choice, micro = best.split("/")[0], built[best][3]
        exch.update(choice=choice, micro_batches=micro, trial_ms_per_step=trials, trial_min_max_ms=spread,
                    rule=("exchange forced by flag; " if forced is not None else "") +
                         f"the lowest median step time of a {Kt}-step trial (after 2 warm-up steps; each step timed "
                         "between a synchronize + barrier, max over ranks) of each exchange x micro-batch count on "
                         "this topology",
                    prediction_agrees=(min(exch["prediction_ms_per_step"], key=exch["prediction_ms_per_step"].get)
                                       == choice) if peak else None)
        fn, t, global_batch, _ = built[best]
        for key in list(built):
            if key != best:
                del built[key]
        torch.cuda.empty_cache()

    # 3. the headline
    wd.phase(f"{topo} x{world}: timing {args.steps} steps",
             PHASE_LIMIT_S["trial"] + 5.0 * (args.steps + args.warmup))
    dt = timed(fn, args.steps, args.warmup, dev)
    out.update(value=args.steps * global_batch / dt, ms_per_step=dt / args.steps * 1e3)
    out["config"] = {"workload": labels[topo], "global_batch": global_batch, "per_gpu_batch": B, "topology": topo,
                     "parallelism": {"pipeline": "k3-client-server", "hub": f"k4-{nc}clients-1server"}.get(topo, f"dp{world}"),
                     "graph": bool(getattr(t, "graph", False))}
    out["scaling"] = "weak"
    step_s = dt / args.steps
    if topo != "replicated":
        out["config"]["micro_batches"] = exch["micro_batches"]
        out["config"]["per_client_batch"] = B
        out["config"]["cut_exchange"] = codec_label[exch["choice"] == "codec"]
        moved, dense = wire(t)
        per_dir_dense = B * CUT_BYTES
        wgbps = moved / 2 / step_s / 1e9
        exch.update(link_bytes_per_step_moved=moved, link_bytes_per_step_dense=dense,
                    cut_bytes_per_link_per_direction_per_step_dense=per_dir_dense,
                    dense_equivalent_GBps_per_link_per_direction=round(per_dir_dense / step_s / 1e9, 2),
                    wire_GBps_per_link_per_direction=round(wgbps, 2),
                    wire_frac_of_measured_p2p_peak=round(wgbps / peak, 3) if peak else None,
                    wire_frac_of_vendor_link=round(wgbps / XGMI_LINK_GBPS, 3))
        if topo == "hub":
            exch["server_inbound_wire_GBps_all_links"] = round(wgbps * nc, 2)
        out["exchange"] = exch
        # the server GPU's roofline over the step, its dominant kernel, and the link beside them
        roof = step_roofline(global_batch / step_s, step_s * 1e3, global_batch)
        roof["link"] = {k: exch[k] for k in ("wire_GBps_per_link_per_direction", "wire_frac_of_measured_p2p_peak",
                                             "wire_frac_of_vendor_link")}
        out["roofline"] = roof
        wd.phase("roofline: server kernel pass", PHASE_LIMIT_S["roofline"])
        try:
            settle()
            dk = [server_kernel_pass(t, B, dev) if rank == world - 1 else None]
            settle()
        except Exception as e:  # noqa: BLE001 (the headline stands on its own)
            dk = [{"error": repr(e)[:300]}]
        dist.broadcast_object_list(dk, src=world - 1)
        out["roofline"]["dominant_kernel"] = dk[0]
    else:
        out["config"]["replica_step"] = ("fused single-GPU step kernels (x3 conv2, client images, client backward "
                                         "in the dgrad epilogue) captured in a HIP graph; bucket all-reduce "
                                         "outside the graph; one launch steps both stages" if t.fused else "unfused")
        roof = step_roofline(B / step_s, step_s * 1e3, B)
        roof["scope"] = "each GPU (replica) over the whole step: " + roof["scope"].split("(", 1)[1].rstrip(")")
        out["roofline"] = roof
    del fn, t
    torch.cuda.empty_cache()

    if topo != "replicated" and not args.no_exchange_phase:
        # side object: data-parallel replicas of the fused K2 step on every GPU (not a BASELINE config)
        wd.phase(f"replicated x{world}: build + {args.exchange_steps} steps", PHASE_LIMIT_S["replicated"])
        try:
            fn2, t2, gb2 = build("replicated", args.micro, False)
            K2 = args.exchange_steps
            dt2 = timed(fn2, K2, 2, dev)
            out["replicated_dp"] = {"workload": labels["replicated"], "samples_per_s": round(K2 * gb2 / dt2, 1),
                                    "ms_per_step": round(dt2 / K2 * 1e3, 3), "global_batch": gb2,
                                    "replica_step": "fused" if t2.fused else "unfused"}
            del fn2, t2
            torch.cuda.empty_cache()
        except Exception as e:  # the headline number stands on its own
            out["replicated_dp"] = {"error": repr(e)[:300]}
    if not args.no_k5:
        # BASELINE config 5 SplitFed: N-1 client GPUs run the widened conv stack, GPU N-1 the head
        wd.phase(f"k5_splitfed x{world}", PHASE_LIMIT_S["k5"])
        try:
            from splitcnn.wide import SyntheticCIFAR, WideClientStage, WideServerStage, init_wide_models
            Bk = args.k5_batch
            wa, wb = init_wide_models(seed=0)
            if rank < world - 1:
                data = SyntheticCIFAR(42 + rank)
                xs, ys = zip(*(data.batch(Bk) for _ in range(2)))
                WX, WY = torch.stack(xs).to(dev), torch.stack(ys).to(dev)
                wt = sd.WideHub(WideClientStage(wa, device=dev), rank, world, client_group=grp, micro=args.micro,
                                groups=groups)
                wfn = lambda i: wt.client_step(WX[i % 2], WY[i % 2])  # noqa: E731
            else:
                wt = sd.WideHub(WideServerStage(wb, device=dev), rank, world, client_group=grp, micro=args.micro,
                                groups=groups)
                wfn = lambda i: wt.server_step(Bk, dev, WideClientStage.cut_shape, WideClientStage.cut_dtype)  # noqa: E731
            Kw = max(3, min(args.steps, 10))
            dtw = timed(wfn, Kw, 2, dev)
            Gw = (world - 1) * Bk
            per_dir = Bk * 32768
            gbps = per_dir / (dtw / Kw) / 1e9
            out["k5_splitfed"] = {
                "workload": f"K5 SplitFed: {world - 1} client GPU(s) (widened conv stack, bf16) + 1 server GPU "
                            f"(dropout/fc/CE head), {args.micro} micro-batches, client all-reduce",
                "samples_per_s": round(Kw * Gw / dtw, 1), "ms_per_step": round(dtw / Kw * 1e3, 3),
                "global_batch": Gw, "per_client_batch": Bk,
                "cut_bytes_per_link_per_direction_per_step": per_dir,
                "exchange_GBps_per_link_per_direction": round(gbps, 2),
                "exchange_frac_of_measured_p2p_peak": round(gbps / peak, 3) if peak else None}
        except Exception as e:
            out["k5_splitfed"] = {"error": repr(e)[:300]}


def progress(msg):
    """Phase marker on stderr (long multi-rank runs stay visibly alive; stdout keeps the one JSON line)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


class Watchdog:
    """Per-phase hang guard of the multi-rank bench (armed by default at N > 1; SLK_BENCH_WATCHDOG=0 turns
    it off, =1 arms it at N = 1 too; SLK_BENCH_WATCHDOG_SCALE multiplies every limit). `phase(name, s)`
    starts a phase that must end within s seconds (the next phase() or disarm() ends it). On expiry the
    watchdog thread dumps every thread's stack to stderr; on rank 0 it prints the JSON line accumulated so
    far (`out`: the headline once measured) with "error": "watchdog: <phase>"; then the process leaves
    with os._exit(3) — no re-launch, and torch.distributed.run then stops the other ranks. Ranks other
    than 0 wait `grace` seconds longer, so that rank 0 (which holds the JSON) reports first.
    SLK_BENCH_STALL=<phase prefix> (+ SLK_BENCH_STALL_RANK, default 0) makes that rank sleep inside the
    first matching phase: the test knob for this path."""

    EXIT_CODE = 3

    def __init__(self, out, rank=0, enabled=True, scale=None, grace=30.0, stream=None):
        self.out, self.rank = out, rank
        self.enabled = bool(enabled)
        self.scale = float(os.environ.get("SLK_BENCH_WATCHDOG_SCALE", "1")) if scale is None else float(scale)
        self.grace = 0.0 if rank == 0 else grace
        self.stream = stream if stream is not None else sys.stdout
        self.name = None
        self.history = []
        self._deadline = None
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._stall = os.environ.get("SLK_BENCH_STALL")
        self._stall_rank = int(os.environ.get("SLK_BENCH_STALL_RANK", "0"))
        if self.enabled:
            threading.Thread(target=self._run, name="slk-bench-watchdog", daemon=True).start()

    def phase(self, name, seconds):
        progress(name)
        with self._lock:
            if self.name is not None:
                self.history.append(self.name)
            self.name = name
            self._deadline = time.monotonic() + seconds * self.scale + self.grace
        if self._stall and name.startswith(self._stall) and self.rank == self._stall_rank:
            self._stall = None
            print(f"[bench] SLK_BENCH_STALL: rank {self.rank} stalls in phase '{name}'", file=sys.stderr, flush=True)
            time.sleep(1e7)

    def disarm(self):
        with self._lock:
            self._deadline = None
        self._stop.set()

    def _run(self):
        while not self._stop.wait(0.25):
            with self._lock:
                late = self._deadline is not None and time.monotonic() > self._deadline
                name = self.name
            if late:
                self._fire(name)

    def _fire(self, name):
        try:
            print(f"[bench] watchdog: phase '{name}' exceeded its limit on rank {self.rank}; all stacks:",
                  file=sys.stderr, flush=True)
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            if self.rank == 0:
                try:
                    o = json.loads(json.dumps(self.out, default=str))   # a snapshot the main thread cannot change
                except Exception:  # noqa: BLE001 (a nested value mutated mid-copy: keep the scalars)
                    o = {k: v for k, v in dict(self.out).items() if isinstance(v, (int, float, str, type(None)))}
                o["error"] = f"watchdog: {name}"
                o["phases_completed"] = list(self.history)
                print(json.dumps(o), file=self.stream, flush=True)
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(self.EXIT_CODE)


def main():
    args = parse()
    if os.environ.get("SLK_BENCH_TRACE_AFTER"):  # debugging aid: dump every thread's stack, then exit
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["SLK_BENCH_TRACE_AFTER"]), exit=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the multi-GPU path on a 1-GPU box: SLK_BENCH_BACKEND=gloo SLK_BENCH_ONE_GPU=1 puts
    # every rank on cuda:0 over gloo (which moves CUDA tensors through the host). Never for numbers.
    backend = os.environ.get("SLK_BENCH_BACKEND", "nccl")
    if os.environ.get("SLK_BENCH_ONE_GPU"):
        local = 0
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    out = {"metric": "training samples/sec (node) for split CNN", "value": None, "unit": "samples/s",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
           "data": "synthetic MNIST-shape batches (class prototypes + noise, normalised (0.1307, 0.3081)), "
                   "random-init weights (seed 0)"}
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_baseline_seconds)  # before this process touches the GPU
    import torch
    import torch.distributed as dist
    wd_env = os.environ.get("SLK_BENCH_WATCHDOG")
    wd = Watchdog(out, rank, enabled=(wd_env != "0") if world > 1 else (wd_env == "1"))
    if world > 1:
        wd.phase("init_process_group", PHASE_LIMIT_S["setup"])
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
        run_distributed(args, out, rank, world, local, wd)
    elif args.config == "k5":
        w = run_wide(args, args.k5_batch, args.steps, args.warmup, not args.no_kernel_pass)
        out.update({k: v for k, v in w.items() if k != "metric"})
        out["metric"] = w["metric"]
        out["data"] = "synthetic CIFAR-shape batches (class prototypes + noise), random-init weights (seed 0)"
    else:
        run_single(args, out)
        if not args.no_hub_loopback:
            try:
                c1 = (out.get("kernels") or {}).get("conv1_fwd")
                out["k4_server_loopback"] = hub_loopback_rate(args, out["value"], c1)
                # the same server step with the dense exchange (no codec kernels on the server; the link
                # then carries 2x the bytes): which one K4 should run depends on the link rate
                import torch
                torch.cuda.empty_cache()
                out["k4_server_loopback"]["dense_exchange"] = {
                    k: v for k, v in hub_loopback_rate(argparse.Namespace(**{**vars(args), "dense_exchange": True}),
                                                       out["value"], c1).items()
                    if k in ("samples_per_s", "ms_per_step", "ratio", "workload")}
                torch.cuda.empty_cache()
                # the dense exchange of the f32 cut (--no-images): the server stages and splits f32 rows
                out["k4_server_loopback"]["dense_f32_cut"] = {
                    k: v for k, v in hub_loopback_rate(argparse.Namespace(**{**vars(args), "dense_exchange": True,
                                                                             "no_images": True}),
                                                       out["value"], c1).items()
                    if k in ("samples_per_s", "ms_per_step", "ratio")}
            except Exception as e:  # the headline stands on its own
                out.setdefault("k4_server_loopback", {})["error"] = repr(e)[:300]
        try:
            import torch
            if not args.no_dropin:
                X, Y = make_pool(args.batch, 4, torch.device("cuda:0"))
                out["dropin_modules"] = run_dropin(X, Y, max(5, min(args.steps, 20)), 3)
                del X, Y
        except Exception as e:  # the headline stands on its own
            out["dropin_modules"] = {"error": repr(e)[:300]}
        if not args.no_k5:
            try:
                out["widened"] = run_wide(args, args.k5_batch, max(5, min(args.steps, 20)), 3,
                                          not args.no_kernel_pass)
            except Exception as e:  # the headline stands on its own
                out["widened"] = {"error": repr(e)[:300]}
    if cpu is not None:
        out["cpu_baseline"] = cpu
        if cpu.get("value"):
            out["speedup_vs_cpu_baseline"] = round(out["value"] / cpu["value"], 1)
    try:
        from splitcnn import _lib
        out["build"] = {"slk_build_id": _lib.build_id()[:16], "variant_defines": _lib.VARIANT_DEFINES}
    except Exception as e:  # noqa: BLE001
        out["build"] = {"error": repr(e)[:200]}
    if world > 1:
        wd.phase("teardown", PHASE_LIMIT_S["teardown"])
        dist.barrier()
    wd.disarm()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
