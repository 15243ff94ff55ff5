"""Profiling only: phase timeline of the fused x3 conv2 dgrad (conv2_dgrad_x3_kernel<true>) from a variant
build with -DSLK_X3D_TRACE=1 (tools/build_variant.sh x3dtrace "-DSLK_X3D_TRACE=1"): per (workgroup, wave,
unit) shader-clock stamps at the unit barrier, around the staging and the MFMA loops and after the
conv1-gradient epilogue. Prints the mean cycles per phase per wave slot.
--kernel wgrad: the same for conv2_wgrad_x3q_kernel (stamps at the unit barrier, after the first-half
waves' dY routing + image DMA issue, after the MFMAs, after the second-half waves' routing).
usage: python tools/x3d_trace.py build_abl/x3dtrace.so [--B 4096] [--kernel dgrad|wgrad]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

NU, NS = 128, 8  # units and stamps per (workgroup, wave) in the probe's buffer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--kernel", default="dgrad", choices=["dgrad", "wgrad", "wgradp"])
    args = ap.parse_args()
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage
    B = args.B
    dev = torch.device("cuda:0")
    a, b = init_models(seed=1)
    x, y = SyntheticMNIST(2).batch(B)
    act = ClientStage(a, device=dev).forward(x.to(dev)).clone()
    xg = x.to(dev).contiguous()
    W1, b1 = a.conv1.weight.detach().to(dev).contiguous(), a.conv1.bias.detach().to(dev).contiguous()
    W2, b2 = b.conv2.weight.detach().to(dev).contiguous(), b.conv2.bias.detach().to(dev).contiguous()
    W3, b3 = b.fc1.weight.detach().to(dev).contiguous(), b.fc1.bias.detach().to(dev).contiguous()
    pooled, code = ops.conv2_fwd_pool(act, W2, b2)
    _, _, _, dp = ops.fc_xent(pooled, W3, b3, y.to(dev), 1.0 / B)
    dpa = ops.row_amax(dp)
    P = ctypes.c_void_p
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L = ctypes.CDLL(os.path.abspath(args.lib), mode=os.RTLD_LOCAL | os.RTLD_DEEPBIND)
    L.slk_conv2_act16_bytes.restype = ctypes.c_int64
    L.slk_conv2_act16_bytes.argtypes = [ctypes.c_int]
    L.slk_conv1_fwd_x3.restype = ctypes.c_int
    L.slk_conv1_fwd_x3.argtypes = [P] * 7 + [ctypes.c_int, P]
    a16 = torch.empty(L.slk_conv2_act16_bytes(B), dtype=torch.uint8, device=dev)
    am1 = torch.empty(B, device=dev)
    bits = torch.empty(B, 768, dtype=torch.int32, device=dev)
    assert L.slk_conv1_fwd_x3(p(xg), p(W1), p(b1), None, p(am1), p(a16), p(bits), B, st) == 0
    L.slk_conv2_dgrad_x3_c1w_nslab.restype = ctypes.c_int
    L.slk_conv2_dgrad_x3_c1w.restype = ctypes.c_int
    L.slk_conv2_dgrad_x3_c1w.argtypes = [P] * 7 + [ctypes.c_int, P]
    sl = torch.empty(L.slk_conv2_dgrad_x3_c1w_nslab(B), 320, device=dev)
    run = lambda: L.slk_conv2_dgrad_x3_c1w(p(dp), p(dpa), p(code), p(W2), p(xg), p(bits), p(sl), B, st)  # noqa: E731
    if args.kernel in ("wgrad", "wgradp"):
        L.slk_conv2_wgrad_x3_nslab.restype = ctypes.c_int
        L.slk_conv2_wgrad_x3s.restype = ctypes.c_int
        L.slk_conv2_wgrad_x3s.argtypes = [P] * 6 + [ctypes.c_int, P]
        slw = torch.empty(L.slk_conv2_wgrad_x3_nslab(B), 18496, device=dev)
        run = lambda: L.slk_conv2_wgrad_x3s(p(a16), p(am1), p(dp), p(dpa), p(code), p(slw), B, st)  # noqa: E731
    ms = []
    for i in range(12):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert run() == 0
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    ms = sorted(ms[2:])
    buf = np.zeros(256 * 8 * NU * NS, dtype=np.uint64)
    rd = L.slk_x3q_trace_read if args.kernel != "dgrad" else L.slk_x3d_trace_read
    assert rd(ctypes.c_void_p(buf.ctypes.data)) == 0
    T = buf.reshape(256, 8, NU, NS).astype(np.int64)
    t_start = T[:, :, 0, 7]
    t_end = T[:, :, 127, 7]
    span = (t_end.max() - t_start.min())
    print(f"kernel median {ms[len(ms) // 2]:.4f} ms; stamp span {span} ticks -> {span / (ms[len(ms) // 2] * 1e3):.1f} ticks/us")
    G = 256
    if args.kernel == "wgrad":
        wgrad_report(T, (6 * B + G - 1) // G)
        return
    if args.kernel == "wgradp":  # the sparse wgrad: 3 units per sample, nslab = min(6 B, 256) K shares
        per = (3 * B + G - 1) // G
        wgrad_report(T, per)
        return
    per = (3 * B + G - 1) // G
    nu = 2 * per
    print(f"units per workgroup {nu}")
    pro = (T[:, :, 1, 7] - T[:, :, 0, 7]).mean()
    init = (T[:, :, 2, 7] - T[:, :, 1, 7]).mean()
    tail_end = (T[:, :, 127, 7] - np.maximum(T[:, :, nu - 1, 5], T[:, :, nu - 1, 4])).mean()
    first_wait = (T[:, :, 0, 6] - T[:, :, 2, 7]).mean()
    print(f"prologue (W2 load/split) {pro:.0f}  first staging {init:.0f}  to first barrier {first_wait:.0f}  "
          f"after last unit {tail_end:.0f}")
    wg_span = (T[:, :, 127, 7].max(1) - T[:, :, 0, 7].min(1))
    print(f"workgroup span: mean {wg_span.mean():.0f} min {wg_span.min()} max {wg_span.max()}; "
          f"start skew {t_start.min(1).max() - t_start.min()}  end skew {t_end.max() - t_end.max(1).min()}")
    u = np.arange(nu)
    bar = T[:, :, u, 0] - T[:, :, u, 6]
    pre = T[:, :, u, 1] - T[:, :, u, 0]
    main_ = T[:, :, u, 2] - T[:, :, u, 1]
    post = T[:, :, u, 3] - T[:, :, u, 2]
    t3 = T[:, :, u, 4] - T[:, :, u, 3]
    epi = np.where(u % 2 == 1, T[:, :, u, 5] - T[:, :, u, 4], 0)
    endu = np.where(u % 2 == 1, T[:, :, u, 5], T[:, :, u, 4])
    gap = np.zeros_like(bar)
    gap[:, :, :-1] = T[:, :, u[1:], 6] - endu[:, :, :-1]
    unit = np.zeros_like(bar)
    unit[:, :, :-1] = T[:, :, u[1:], 0] - T[:, :, u[:-1], 0]
    print("per unit, mean cycles over workgroups and units (wave = nt + 2 g; waves 4-7 stage first)")
    print(f"{'wave':>4} {'barrier':>8} {'stage<':>8} {'mfma27':>8} {'stage>':>8} {'tile3':>8} {'epi(h1)':>8} {'gap':>6} {'unit':>8}")
    for w in range(8):
        print(f"{w:>4} {bar[:, w].mean():8.0f} {pre[:, w].mean():8.0f} {main_[:, w].mean():8.0f} {post[:, w].mean():8.0f} "
              f"{t3[:, w].mean():8.0f} {epi[:, w, 1::2].mean():8.0f} {gap[:, w, :-1].mean():6.0f} {unit[:, w, :-1].mean():8.0f}")
    # by part (pair index -> part), h
    p0 = np.minimum(np.arange(G) * per, 3 * B)
    for pt in range(3):
        for h in range(2):
            sel = [(wg, uu) for wg in range(G) for uu in range(nu - 1) if uu % 2 == h and ((p0[wg] + uu // 2) % 3) == pt]
            if not sel:
                continue
            wgs, uus = np.array(sel).T
            print(f"part {pt} h {h}: unit {unit[wgs, :, uus].mean():7.0f}  barrier wait by wave "
                  + " ".join(f"{bar[wgs, w, uus].mean():5.0f}" for w in range(8))
                  + "  mfma by wave " + " ".join(f"{(main_ + t3)[wgs, w, uus].mean():5.0f}" for w in range(8)))


def wgrad_report(T, nu):
    u = np.arange(nu)
    print(f"units per workgroup {nu}; prologue {(T[:, :, 0, 0] - T[:, :, 0, 7]).mean():.0f}")
    bar = T[:, :, u, 0] - T[:, :, u, 6]
    pre = T[:, :, u, 1] - T[:, :, u, 0]
    mf = T[:, :, u, 2] - T[:, :, u, 1]
    post = T[:, :, u, 3] - T[:, :, u, 2]
    gap = np.zeros_like(bar)
    gap[:, :, :-1] = T[:, :, u[1:], 6] - T[:, :, u[:-1], 3]
    unit = np.zeros_like(bar)
    unit[:, :, :-1] = T[:, :, u[1:], 0] - T[:, :, u[:-1], 0]
    dwait = np.zeros_like(bar)
    sto = np.zeros_like(bar)
    if T[:, :, u, 4].any():  # the sparse kernel's stamps inside its staging: data ready (4), stores done (5)
        first = np.where(np.arange(8)[None, :, None] >= 4, T[:, :, u, 0], T[:, :, u, 2])
        dwait = T[:, :, u, 4] - first
        sto = T[:, :, u, 5] - T[:, :, u, 4]
        print("staging: cycles from its start to its data (the loads' wait) and then to its last store, by wave")
        for w in range(8):
            print(f"{w:>4} wait {dwait[:, w].mean():8.0f}  stores {sto[:, w].mean():8.0f}")
    print("wave = 4 tg + 2 c + h; tg 1 (waves 4-7) route before their MFMAs; waves 6-7 route nothing")
    print(f"{'wave':>4} {'barrier':>8} {'route<':>8} {'mfma':>8} {'route>':>8} {'gap':>6} {'unit':>8}")
    for w in range(8):
        print(f"{w:>4} {bar[:, w].mean():8.0f} {pre[:, w].mean():8.0f} {mf[:, w].mean():8.0f} {post[:, w].mean():8.0f} "
              f"{gap[:, w, :-1].mean():6.0f} {unit[:, w, :-1].mean():8.0f}")


if __name__ == "__main__":
    main()
