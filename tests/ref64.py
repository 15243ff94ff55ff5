"""Test infrastructure: float64 references of conv2 (src/model_def.py:18,25-27) evaluated on the GPU with
torch float64 GEMMs (unfold + matmul: no MIOpen, no reduced precision), so full-size (B = 4096)
parity checks finish in seconds. Same semantics as oracle/split_step.py (conv3x3 / conv3x3_dgrad /
conv3x3_wgrad / maxpool2_bwd / tie_discrepancies), restated in torch for batch throughput."""
import torch
import torch.nn.functional as F



def conv_relu64(act, W2, b2):
    """relu(conv2d(act, W2, b2)) in float64: act [B,32,26,26] -> [B,64,24,24]."""
    B = act.shape[0]
    cols = F.unfold(act.double(), 3)                                   # B, 288, 576
    y = torch.matmul(W2.double().reshape(64, 288), cols) + b2.double()[None, :, None]
    return y.reshape(B, 64, 24, 24).clamp_min(0.0)


def route64(dpooled, code):
    """max-pool + ReLU backward by the kernels' routing code (0-3 = argmax position, 4 = blocked):
    dc [B,64,24,24] float64 (oracle.split_step.maxpool2_bwd on the routed values)."""
    B = code.shape[0]
    dp = dpooled.double().reshape(B, 64, 12, 12)
    c = code.long()
    d = torch.zeros(B, 64, 12, 12, 4, dtype=torch.float64, device=dp.device)
    d.scatter_(-1, c.clamp_max(3)[..., None], torch.where(c < 4, dp, torch.zeros_like(dp))[..., None])
    return d.reshape(B, 64, 12, 12, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, 64, 24, 24)


def dgrad64(dc, W2):
    """cut gradient = full correlation of dc with W2: [B,64,24,24] -> [B,32,26,26] float64."""
    B = dc.shape[0]
    cols = torch.matmul(W2.double().reshape(64, 288).t(), dc.reshape(B, 64, 576))   # B, 288, 576
    return F.fold(cols, (26, 26), 3)


def wgrad64(act, dc, chunk=512):
    """dW2 [64,32,3,3] and db2 [64] in float64, summed over the batch in chunks."""
    dW = torch.zeros(64, 288, dtype=torch.float64, device=dc.device)
    for s in range(0, act.shape[0], chunk):
        cols = F.unfold(act[s:s + chunk].double(), 3)                  # b, 288, 576
        d = dc[s:s + chunk].reshape(-1, 64, 576)
        dW += torch.matmul(d, cols.transpose(1, 2)).sum(0)
    return dW.reshape(64, 32, 3, 3), dc.sum(dim=(0, 2, 3))


def routing64(r):
    """The kernels' routing code from a float64 relu'd conv output [B,64,24,24] (oracle.split_step.maxpool2
    + route_code: first max wins, strict >; 4 where the pooled value is <= 0) and the windows [B,64,12,12,4]."""
    B = r.shape[0]
    win = r.reshape(B, 64, 12, 2, 12, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, 64, 12, 12, 4)
    best = win[..., 0].clone()
    idx = torch.zeros(best.shape, dtype=torch.long, device=r.device)
    for q in range(1, 4):
        bt = win[..., q] > best
        best = torch.where(bt, win[..., q], best)
        idx = torch.where(bt, torch.full_like(idx, q), idx)
    return torch.where(best > 0, idx, torch.full_like(idx, 4)), win


def assert_routing_ties(act, W2, b2, code, chunk=512, rtol=1e-5, atol=1e-6):
    """Every window where the kernel's routing code (uint8 [B,64,12,12]) differs from float64's must be a
    numerical tie: the two candidates' float64 values (0 for a ReLU-blocked code) within
    max(rtol * |window max|, atol * max|r|). atol is the f32 conv's own absolute error against float64
    (measured 4-5e-7 of max|r| for the x3 and the direct f32 kernels at B = 4096), which decides windows at
    the ReLU boundary, e.g. a max of 1e-7 that one path rounds to <= 0. Checked for EVERY window of every
    sample (float64 conv on the GPU). Returns the number of differing windows."""
    B = act.shape[0]
    scale = 0.0
    rs = []
    for s in range(0, B, chunk):
        r = conv_relu64(act[s:s + chunk], W2, b2)
        scale = max(scale, r.abs().max().item())
        rs.append(r)
    n = 0
    for s, r in zip(range(0, B, chunk), rs):
        c64, win = routing64(r)
        c = code[s:s + chunk].long()
        d = c != c64
        k = int(d.sum())
        if not k:
            continue
        n += k
        w = win[d]
        mx = w.max(-1).values
        va = torch.where(c[d] < 4, w.gather(-1, c[d].clamp_max(3)[:, None])[:, 0], torch.zeros_like(mx))
        vb = torch.where(c64[d] < 4, w.gather(-1, c64[d].clamp_max(3)[:, None])[:, 0], torch.zeros_like(mx))
        tol = torch.maximum(rtol * mx.abs(), torch.full_like(mx, atol * scale))
        bad = (va - vb).abs() > tol
        assert not bad.any(), (f"{int(bad.sum())} of {k} routing differences from float64 are not ties: gaps/scale "
                               f"{((va - vb).abs()[bad] / scale).tolist()[:6]}, window max/scale {(mx[bad] / scale).tolist()[:6]}")
    return n
