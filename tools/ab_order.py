"""Profiling-only: the fused split step with the server/client backward kernels in different (all
dependency-respecting) orders, each captured as a HIP graph, timed interleaved in ONE process.
Tokens: dg = conv2 dgrad, wg = conv2 wgrad, fw = fc wgrad, S = server SGD + loss log (after dg, wg,
fw: dg reads W2), c1 = client wgrad (after dg), C = client SGD (after c1).
usage: python tools/ab_order.py"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]
from bench import make_pool  # noqa: E402
from splitcnn import ops  # noqa: E402
from splitcnn.data import init_models  # noqa: E402
from splitcnn.engine import SplitTrainer  # noqa: E402

ORDERS = os.environ.get("ORDERS", "dg,wg,fw,S,c1,C;fw,dg,wg,S,c1,C;wg,dg,fw,S,c1,C;fw,wg,dg,S,c1,C;"
                                  "dg,fw,wg,S,c1,C;wg,fw,dg,S,c1,C;dg,c1,wg,fw,S,C;dg,wg,fw,c1,S,C").split(";")
B, K, R = 4096, 20, 6
dev = torch.device("cuda:0")
X, Y = make_pool(B, 4, dev)


def make_step(order, tr):
    c, s = tr.client, tr.server
    m = s.model
    W2, b2 = m.conv2.weight.detach(), m.conv2.bias.detach()
    W3, b3 = m.fc1.weight.detach(), m.fc1.bias.detach()
    k = ops.CONV2_SLAB

    def step(x, y):
        act = c.forward(x)
        pooled, code = ops.conv2_fwd_pool(act, W2, b2, pooled=s._b("pooled", (B, 64, 12, 12)),
                                          code=s._b("code", (B, 64, 12, 12), torch.uint8))
        _, loss_i, dlogits, dpooled = ops.fc_xent(
            pooled, W3, b3, y, 1.0 / B, logits=s._b("logits", (B, 10)), loss_i=s._b("loss_i", (B,)),
            dlogits=s._b("dlogits", (B, 10)), dpooled=s._b("dpooled", (B, 64, 12, 12)), err_flag=s.err_flag)
        cut = s._b("cut_grad", (B, 32, 26, 26))
        s2 = s._b("s2", (ops.conv2_wgrad_nslab(B), ops.CONV2_SLAB))
        s3 = s._b("s3", (ops.fc_wgrad_nslab(B), ops.FC_SLAB))
        s1 = c._buf.get("slabs", (ops.conv1_wgrad_nslab(B), ops.CLIENT_NPARAM), torch.float32, dev)
        for t in order:
            if t == "dg":
                ops.conv2_dgrad(dpooled, code, W2, out=cut)
            elif t == "wg":
                ops.conv2_wgrad_slabs(act, dpooled, code, slabs=s2)
            elif t == "fw":
                ops.fc_wgrad_slabs(dlogits, pooled, slabs=s3)
            elif t == "S":
                ops.sgd_multi_from_slabs([(s.params[:k], s.grads[:k], s2), (s.params[k:], s.grads[k:], s3)], s.lr,
                                         loss=(loss_i, 1.0 / B, s.loss_log.ring, s.loss_log.counter))
            elif t == "c1":
                ops.conv1_wgrad_remask_slabs(x, c.W1.detach(), c.b1.detach(), cut, slabs=s1)
            elif t == "C":
                ops.sgd_from_slabs(c.params, c.grads, s1, c.lr)
    return step


variants = {}
for o in ORDERS:
    tr = SplitTrainer(*init_models(seed=0), device=dev, graph=False)
    fn = make_step(o.split(","), tr)
    xs = torch.zeros_like(X[0])
    ys = torch.zeros_like(Y[0])
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(st):
        fn(xs, ys)
    torch.cuda.current_stream(dev).wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn(xs, ys)
    variants[o] = (g, xs, ys, tr)
res = {k: [] for k in variants}
for r in range(R):
    for o, (g, xs, ys, tr) in variants.items():
        for i in range(3):
            xs.copy_(X[i % 4]); ys.copy_(Y[i % 4]); g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            xs.copy_(X[i % 4]); ys.copy_(Y[i % 4]); g.replay()
        torch.cuda.synchronize()
        res[o].append((time.perf_counter() - t0) / K * 1e3)
# same final weights for every order (the orders only permute independent launches)
ref = None
for o, (g, xs, ys, tr) in variants.items():
    w = torch.cat([tr.client.params, tr.server.params])
    print(json.dumps({"order": o, "min_ms": round(min(res[o]), 4), "median_ms": round(sorted(res[o])[R // 2], 4),
                      "same_weights_as_first": bool(ref is None or torch.equal(ref, w))}))
    ref = w if ref is None else ref
