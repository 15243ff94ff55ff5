"""Profiling only: the x3 conv2 kernels of several libslk builds (tools/build_variant.sh outputs) timed
side by side in ONE process, interleaved rounds, HIP events on one stream, B = 4096, real activations.
usage: python tools/x3_ab.py lib0.so lib1.so ... [--rounds 30] [--ops fwd,dgrad,wgrad]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--flush", action="store_true",
                    help="read 600 MB before every timed call (outside the timing): operands come from HBM, "
                         "not the 256 MB Infinity Cache, as inside the step")
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
    xg = x.to(dev).contiguous()
    W1, b1 = a.conv1.weight.detach().to(dev).contiguous(), a.conv1.bias.detach().to(dev).contiguous()
    W2, b2 = b.conv2.weight.detach().to(dev).contiguous(), b.conv2.bias.detach().to(dev).contiguous()
    W3, b3 = b.fc1.weight.detach().to(dev).contiguous(), b.fc1.bias.detach().to(dev).contiguous()
    amax = ops.row_amax(act)
    pooled, code = ops.conv2_fwd_pool(act, W2, b2)
    _, _, _, dp = ops.fc_xent(pooled, W3, b3, y.to(dev), 1.0 / B)
    dpa = ops.row_amax(dp)
    a16 = torch.empty(ops.conv2_act16_bytes(B), dtype=torch.uint8, device=dev)
    ops.conv2_fwd_pool(act, W2, b2, impl="x3", act_amax=amax, act16=a16)
    P = ctypes.c_void_p
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    if "unp" in args.ops.split(",") or "dgp" in args.ops.split(","):  # the codec's packed form of act (mask, values, word ranks)
        from splitcnn.codec import CutCodec
        cc = CutCodec()
        nel = act.numel()
        cbk = cc.buffers("ab", nel, dev)
        cc.encode(act, cbk)
        crk = cc.ranks("ab", nel, cbk)
        print("unp: set fraction", round(int(cbk[3].item()) / nel, 4), flush=True)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cases = {}
    outs = {}  # case -> output tensor (compared across libraries after the timing)
    for li, path in enumerate(args.libs):
        L = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL | os.RTLD_DEEPBIND)  # own symbols first
        for n in ("slk_conv2_fwd_pool_x3s", "slk_conv2_dgrad_x3", "slk_conv2_wgrad_x3s", "slk_conv2_wgrad_x3_nslab"):
            getattr(L, n).restype = ctypes.c_int
        tag = os.path.basename(path).replace(".so", "")
        # this library's own act16 images (layouts may differ between builds)
        L.slk_conv2_act16_bytes.restype = ctypes.c_int64
        L.slk_conv2_act16_bytes.argtypes = [ctypes.c_int]
        # ABI 2 (round 3): conv1_fwd_x3 also writes the ReLU bit map, the fused dgrad reads it instead of
        # W1 / b1; older builds (ABI 1) are driven with their own argument lists
        abi2 = hasattr(L, "slk_relu_bits_bytes")
        L.slk_conv1_fwd_x3.restype = ctypes.c_int
        L.slk_conv1_fwd_x3.argtypes = [P] * (7 if abi2 else 6) + [ctypes.c_int, P]
        a16 = torch.empty(L.slk_conv2_act16_bytes(B), dtype=torch.uint8, device=dev)
        am1 = torch.empty(B, device=dev)
        bits = torch.empty(B, 768, dtype=torch.int32, device=dev)
        c1x = (lambda L, am, img: L.slk_conv1_fwd_x3(p(xg), p(W1), p(b1), None, p(am), p(img), p(bits), B, st)) if abi2 \
            else (lambda L, am, img: L.slk_conv1_fwd_x3(p(xg), p(W1), p(b1), None, p(am), p(img), B, st))
        assert c1x(L, am1, a16) == 0
        if "c1x3" in args.ops:
            i1 = torch.empty_like(a16)
            cases[f"c1x3 {tag}"] = (lambda L=L, am1=am1, i1=i1, f=c1x: f(L, am1, i1))
            outs[f"c1x3 {tag}"] = i1
        dgc1_args = (lambda: (p(xg), p(bits))) if abi2 else (lambda: (p(xg), p(W1), p(b1)))
        if "fwd," in args.ops + "," :
            po, co, a16o = torch.empty_like(pooled), torch.empty_like(code), torch.empty_like(a16)
            L.slk_conv2_fwd_pool_x3s.argtypes = [P] * 7 + [ctypes.c_int, P]
            cases[f"fwd {tag}"] = (lambda L=L, po=po, co=co, a16o=a16o: L.slk_conv2_fwd_pool_x3s(
                p(act), p(amax), p(W2), p(b2), p(po), p(co), p(a16o), B, st))
        if "unp" in args.ops.split(","):
            L.slk_cut_unpack_x3.restype = ctypes.c_int
            L.slk_cut_unpack_x3.argtypes = [P] * 4 + [ctypes.c_int, P, P]
            iu = torch.empty_like(a16)
            cases[f"unp {tag}"] = (lambda L=L, iu=iu: L.slk_cut_unpack_x3(p(cbk[4]), p(cbk[0]), p(crk), p(amax), B, p(iu), st))
            outs[f"unp {tag}"] = iu
        if "fwdsa" in args.ops and hasattr(L, "slk_conv2_fwd_pool_x3sa"):
            po3, co3, a16s, ams = torch.empty_like(pooled), torch.empty_like(code), torch.empty_like(a16), torch.empty_like(amax)
            L.slk_conv2_fwd_pool_x3sa.restype = ctypes.c_int
            L.slk_conv2_fwd_pool_x3sa.argtypes = [P] * 7 + [ctypes.c_int, P]
            cases[f"fwdsa {tag}"] = (lambda L=L, po=po3, co=co3, a16o=a16s, ams=ams: L.slk_conv2_fwd_pool_x3sa(
                p(act), p(ams), p(W2), p(b2), p(po), p(co), p(a16o), B, st))
            outs[f"fwdsa {tag}"] = po3
        if "fwdi" in args.ops:
            po2, co2 = torch.empty_like(pooled), torch.empty_like(code)
            L.slk_conv2_fwd_pool_x3i.restype = ctypes.c_int
            L.slk_conv2_fwd_pool_x3i.argtypes = [P] * 6 + [ctypes.c_int, P]
            cases[f"fwdi {tag}"] = (lambda L=L, po=po2, co=co2, a16=a16: L.slk_conv2_fwd_pool_x3i(
                p(a16), p(amax), p(W2), p(b2), p(po), p(co), B, st))
            outs[f"fwdi {tag}"] = po2
        if "dgrad" in args.ops:
            g = torch.empty_like(act)
            L.slk_conv2_dgrad_x3.argtypes = [P] * 5 + [ctypes.c_int, P]
            cases[f"dgrad {tag}"] = (lambda L=L, g=g: L.slk_conv2_dgrad_x3(p(dp), p(dpa), p(code), p(W2), p(g), B, st))
            outs[f"dgrad {tag}"] = g
        if "dgp" in args.ops.split(",") and hasattr(L, "slk_conv2_dgrad_x3_pack"):
            gv = torch.empty(act.numel(), device=dev)
            L.slk_conv2_dgrad_x3_pack.restype = ctypes.c_int
            L.slk_conv2_dgrad_x3_pack.argtypes = [P] * 7 + [ctypes.c_int, P]
            cases[f"dgp {tag}"] = (lambda L=L, gv=gv: L.slk_conv2_dgrad_x3_pack(
                p(dp), p(dpa), p(code), p(W2), p(cbk[0]), p(crk), p(gv), B, st))
            outs[f"dgp {tag}"] = gv
        if "dgc1" in args.ops:
            sl1 = torch.empty(L.slk_conv2_dgrad_x3_c1w_nslab(B), 320, device=dev)
            L.slk_conv2_dgrad_x3_c1w.restype = ctypes.c_int
            L.slk_conv2_dgrad_x3_c1w_nslab.restype = ctypes.c_int
            L.slk_conv2_dgrad_x3_c1w.argtypes = [P] * (7 if abi2 else 8) + [ctypes.c_int, P]
            cases[f"dgc1 {tag}"] = (lambda L=L, sl=sl1, xa=dgc1_args(): L.slk_conv2_dgrad_x3_c1w(
                p(dp), p(dpa), p(code), p(W2), *xa, p(sl), B, st))
            outs[f"dgc1 {tag}"] = sl1
        if "fc" in args.ops.split(","):
            lg, li, dlg, dpo, dpam = (torch.empty(B, 10, device=dev), torch.empty(B, device=dev),
                                     torch.empty(B, 10, device=dev), torch.empty_like(dp), torch.empty(B, device=dev))
            yl = y.to(dev)
            L.slk_fc_xent_amax.restype = ctypes.c_int
            L.slk_fc_xent_amax.argtypes = [P] * 9 + [ctypes.c_float, P, ctypes.c_int, P]
            cases[f"fc {tag}"] = (lambda L=L, lg=lg, li=li, dlg=dlg, dpo=dpo, dpam=dpam, yl=yl: L.slk_fc_xent_amax(
                p(pooled), p(W3), p(b3), p(yl), p(lg), p(li), p(dlg), p(dpo), p(dpam), 1.0 / B, None, B, st))
            outs[f"fc {tag}"] = dpo
        if "fc3" in args.ops.split(","):  # the same head as three launches: logits, CE, dpooled
            lg3, li3, dl3, dpo3 = (torch.empty(B, 10, device=dev), torch.empty(B, device=dev),
                                   torch.empty(B, 10, device=dev), torch.empty_like(dp))
            yl3 = y.to(dev)
            for n in ("slk_fc_fwd", "slk_xent_fwd_bwd", "slk_fc_dgrad"):
                getattr(L, n).restype = ctypes.c_int
            L.slk_fc_fwd.argtypes = [P] * 4 + [ctypes.c_int, P]
            L.slk_xent_fwd_bwd.argtypes = [P] * 4 + [ctypes.c_float, P, ctypes.c_int, P]
            L.slk_fc_dgrad.argtypes = [P] * 3 + [ctypes.c_int, P]
            cases[f"fc3 {tag}"] = (lambda L=L, lg=lg3, li=li3, dl=dl3, dpo=dpo3, yl=yl3: L.slk_fc_fwd(
                p(pooled), p(W3), p(b3), p(lg), B, st) | L.slk_xent_fwd_bwd(p(lg), p(yl), p(li), p(dl), 1.0 / B, None, B, st)
                | L.slk_fc_dgrad(p(dl), p(W3), p(dpo), B, st))
            cases[f"fc1 {tag}"] = (lambda L=L, lg=lg3: L.slk_fc_fwd(p(pooled), p(W3), p(b3), p(lg), B, st))
            cases[f"fc4 {tag}"] = (lambda L=L, dl=dl3, dpo=dpo3: L.slk_fc_dgrad(p(dl), p(W3), p(dpo), B, st))
            outs[f"fc {tag}3"] = dpo3
            outs[f"fcl {tag}"] = lg3
        if "fcord" in args.ops.split(","):
            # launch order of the server head + fc weight gradient: A = the step's (fused head, then
            # fc_wgrad: pooled evicted by the head's own 151 MB dpooled write); B = logits, CE, fc_wgrad
            # (pooled re-read while still in the Infinity Cache), dpooled last
            for n in ("slk_fc_fwd", "slk_xent_fwd_bwd", "slk_fc_dgrad", "slk_fc_wgrad", "slk_fc_xent_amax",
                      "slk_fc_wgrad_nslab"):
                getattr(L, n).restype = ctypes.c_int
            L.slk_fc_fwd.argtypes = [P] * 4 + [ctypes.c_int, P]
            L.slk_xent_fwd_bwd.argtypes = [P] * 4 + [ctypes.c_float, P, ctypes.c_int, P]
            L.slk_fc_dgrad.argtypes = [P] * 3 + [ctypes.c_int, P]
            L.slk_fc_wgrad.argtypes = [P] * 3 + [ctypes.c_int, P]
            L.slk_fc_xent_amax.argtypes = [P] * 9 + [ctypes.c_float, P, ctypes.c_int, P]
            yo = y.to(dev)
            oA = [torch.empty(B, 10, device=dev), torch.empty(B, device=dev), torch.empty(B, 10, device=dev),
                  torch.empty_like(dp), torch.empty(B, device=dev), torch.empty(L.slk_fc_wgrad_nslab(B), 92170, device=dev)]
            oB = [torch.empty_like(t) for t in oA]
            cases[f"fcA {tag}"] = (lambda L=L, o=oA: L.slk_fc_xent_amax(
                p(pooled), p(W3), p(b3), p(yo), p(o[0]), p(o[1]), p(o[2]), p(o[3]), p(o[4]), 1.0 / B, None, B, st)
                | L.slk_fc_wgrad(p(o[2]), p(pooled), p(o[5]), B, st))
            cases[f"fcB {tag}"] = (lambda L=L, o=oB: L.slk_fc_fwd(p(pooled), p(W3), p(b3), p(o[0]), B, st)
                | L.slk_xent_fwd_bwd(p(o[0]), p(yo), p(o[1]), p(o[2]), 1.0 / B, None, B, st)
                | L.slk_fc_wgrad(p(o[2]), p(pooled), p(o[5]), B, st) | L.slk_fc_dgrad(p(o[2]), p(W3), p(o[3]), B, st))
            cases[f"fcwA {tag}"] = (lambda L=L, o=oA: L.slk_fc_wgrad(p(o[2]), p(pooled), p(o[5]), B, st))
        if "fch" in args.ops.split(","):  # the step's head launches: logits + CE (one launch), dpooled (+ dp_amax)
            L.slk_fc_logits_xent.restype = ctypes.c_int
            L.slk_fc_logits_xent.argtypes = [P] * 7 + [ctypes.c_float, P, ctypes.c_int, P]
            L.slk_fc_dgrad_amax.restype = ctypes.c_int
            L.slk_fc_dgrad_amax.argtypes = [P] * 4 + [ctypes.c_int, P]
            yo = y.to(dev)
            oh = [torch.empty(B, 10, device=dev), torch.empty(B, device=dev), torch.empty(B, 10, device=dev),
                  torch.empty_like(dp), torch.empty(B, device=dev)]
            cases[f"fch3 {tag}"] = (lambda L=L, o=oh: L.slk_fc_logits_xent(p(pooled), p(W3), p(b3), p(yo), p(o[0]), p(o[1]),
                                                                          p(o[2]), 1.0 / B, None, B, st))
            cases[f"fch4 {tag}"] = (lambda L=L, o=oh: L.slk_fc_dgrad_amax(p(o[2]), p(W3), p(o[3]), p(o[4]), B, st))
            outs[f"fch3 {tag}"] = oh[0]
            outs[f"fch4 {tag}"] = oh[3]
        if "fcw" in args.ops.split(","):
            L.slk_fc_wgrad_nslab.restype = ctypes.c_int
            L.slk_fc_wgrad.restype = ctypes.c_int
            L.slk_fc_wgrad.argtypes = [P] * 3 + [ctypes.c_int, P]
            dlw = torch.randn(B, 10, device=dev, generator=torch.Generator(device=dev).manual_seed(5)) / B
            slw = torch.empty(L.slk_fc_wgrad_nslab(B), 92170, device=dev)
            cases[f"fcw {tag}"] = (lambda L=L, dlw=dlw, slw=slw: L.slk_fc_wgrad(p(dlw), p(pooled), p(slw), B, st))
            outs[f"fcw {tag}"] = slw
        if "wgradf" in args.ops.split(","):  # the f32-act entry (forward images not shared)
            slf = torch.zeros(L.slk_conv2_wgrad_x3_nslab(B), ops.CONV2_SLAB, device=dev)
            L.slk_conv2_wgrad_x3.argtypes = [P] * 6 + [ctypes.c_int, P]
            cases[f"wgradf {tag}"] = (lambda L=L, sl=slf: L.slk_conv2_wgrad_x3(p(act), p(amax), p(dp), p(dpa), p(code), p(sl), B, st))
            outs[f"wgradf {tag}"] = slf
        if "wgrad" in args.ops.split(","):
            sl = torch.empty(L.slk_conv2_wgrad_x3_nslab(B), ops.CONV2_SLAB, device=dev)
            L.slk_conv2_wgrad_x3s.argtypes = [P] * 6 + [ctypes.c_int, P]
            cases[f"wgrad {tag}"] = (lambda L=L, sl=sl, a16=a16: L.slk_conv2_wgrad_x3s(p(a16), p(amax), p(dp), p(dpa), p(code), p(sl), B, st))
            outs[f"wgrad {tag}"] = sl
    times = {k: [] for k in cases}
    for _ in range(3):
        for f in cases.values():
            assert f() == 0
    torch.cuda.synchronize()
    # a READ of 600 MB evicts with clean lines (a write would leave dirty ones the next kernel pays for)
    flushbuf = torch.ones(150_000_000, device=dev) if args.flush else None
    flushout = torch.empty((), device=dev) if args.flush else None
    for _ in range(args.rounds):
        for k, f in cases.items():
            if flushbuf is not None:
                torch.sum(flushbuf, dim=0, out=flushout)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1))
    for k, v in sorted(times.items()):
        v.sort()
        print(f"{k:24s} median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f}", flush=True)
    first = {}
    for k, t in outs.items():  # each library's output vs the first library's (same op)
        op = k.split()[0]
        if op not in first:
            first[op] = t
            continue
        r = first[op]
        red = (lambda z: z.sum(0)) if op in ("dgc1", "fcw", "wgrad", "wgradf") else (lambda z: z)
        a, b_ = red(t.double()), red(r.double())
        print(f"check {k:18s} max|diff|/max|ref| {((a - b_).abs().max() / b_.abs().max()).item():.3e}", flush=True)


if __name__ == "__main__":
    main()
