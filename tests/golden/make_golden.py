"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run in the build container (where /root/reference exists):  python tests/golden/make_golden.py

It imports the reference's own src/model_def.py (ModelPartA/ModelPartB/FullModel, read-only, no
bytecode written) and drives it with the reference's step semantics:
  client: optimizer.zero_grad(); activations = model(data)                    client_part.py:112-114
          payload = activations.clone().detach()                              client_part.py:118
  server: act.requires_grad_(True); optimizer.zero_grad(); outputs = model(act);
          loss = CrossEntropyLoss()(outputs, labels); loss.backward(); optimizer.step()
          cut_grad = act.grad.clone().detach()                                server_part.py:45-57
  client: activations.backward(cut_grad); optimizer.step()                    client_part.py:132-133
with optim.SGD(lr=0.01) on both sides (client_part.py:17, server_part.py:15). client_part.py and
server_part.py themselves are not importable offline (torchvision / mlflow / boto3 are absent and
both contact the cluster at import), so their 20 lines of step logic are restated here.

The fixtures hold inputs and expected outputs only (npz of float32/int64 arrays). The reference
source never leaves /root/reference.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
REF_SRC = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "split-learning-k8s_amd"))

from splitcnn.data import SyntheticMNIST  # noqa: E402  (our seeded synthetic batches)

PARAM_KEYS = [("W1", "conv1.weight"), ("b1", "conv1.bias"), ("W2", "conv2.weight"),
              ("b2", "conv2.bias"), ("W3", "fc1.weight"), ("b3", "fc1.bias")]


def ref_model_def():
    sys.path.insert(0, REF_SRC)
    import model_def  # the reference module
    sys.path.pop(0)
    return model_def


class RefSplit:
    """The reference's two processes, in one: client ModelPartA + server ModelPartB."""

    def __init__(self, md, seed):
        torch.manual_seed(seed)
        self.client = md.ModelPartA()
        self.server = md.ModelPartB()
        self.copt = torch.optim.SGD(self.client.parameters(), lr=0.01)
        self.sopt = torch.optim.SGD(self.server.parameters(), lr=0.01)
        self.crit = torch.nn.CrossEntropyLoss()

    def params(self):
        sd = {**self.client.state_dict(), **self.server.state_dict()}
        return {k: sd[n].detach().numpy().copy() for k, n in PARAM_KEYS}

    def grads(self):
        named = dict(list(self.client.named_parameters()) + list(self.server.named_parameters()))
        return {k: named[n].grad.detach().numpy().copy() for k, n in PARAM_KEYS}

    def step(self, x, y):
        self.copt.zero_grad()
        activations = self.client(x)
        act = activations.clone().detach()
        act.requires_grad_(True)
        self.sopt.zero_grad()
        outputs = self.server(act)
        loss = self.crit(outputs, y)
        loss.backward()
        self.sopt.step()
        cut_grad = act.grad.clone().detach()
        activations.backward(cut_grad)
        self.copt.step()
        return dict(act=act.detach().numpy().copy(), logits=outputs.detach().numpy().copy(),
                    loss=np.float32(loss.item()), cut_grad=cut_grad.numpy().copy())


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


def fixture_steps(md, name, B, nsteps, seed=0, data_seed=42, xform=None, weights_at=(1,)):
    m = RefSplit(md, seed)
    data = SyntheticMNIST(data_seed)
    out = {f"init_{k}": v for k, v in m.params().items()}
    for s in range(1, nsteps + 1):
        x, y = data.batch(B)
        if xform is not None:
            x = xform(x, s)
        r = m.step(x, y)
        out[f"x_{s}"], out[f"y_{s}"] = x.numpy(), y.numpy()
        for k, v in r.items():
            out[f"{k}_{s}"] = v
        if s in weights_at or s == nsteps:
            for k, v in m.params().items():
                out[f"post_{k}_{s}"] = v
            if s == 1:
                for k, v in m.grads().items():
                    out[f"grad_{k}_{s}"] = v
    out["B"], out["nsteps"] = np.int64(B), np.int64(nsteps)
    save(name, **out)


def fixture_curve(md, name, B, nsteps, seed=0, data_seed=42):
    m = RefSplit(md, seed)
    full = None
    data = SyntheticMNIST(data_seed)
    losses = np.zeros(nsteps, dtype=np.float32)
    for s in range(nsteps):
        x, y = data.batch(B)
        losses[s] = m.step(x, y)["loss"]
    out = {"losses": losses, "B": np.int64(B), "nsteps": np.int64(nsteps)}
    for k, v in m.params().items():
        out[f"final_{k}"] = v
    save(name, **out)
    return losses, full


def check_split_equals_full(md, B=64, nsteps=20):
    """a seeded split step equals a seeded FullModel step bit-for-bit."""
    m = RefSplit(md, 0)
    torch.manual_seed(0)
    full = md.FullModel()
    opt = torch.optim.SGD(full.parameters(), lr=0.01)
    crit = torch.nn.CrossEntropyLoss()
    data = SyntheticMNIST(42)
    for _ in range(nsteps):
        x, y = data.batch(B)
        ls = m.step(x, y)["loss"]
        opt.zero_grad()
        lf = crit(full(x), y)
        lf.backward()
        opt.step()
        assert ls == np.float32(lf.item()), (ls, lf.item())
    print("split == full over", nsteps, "steps")


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    md = ref_model_def()
    if sys.argv[1:] == ["b14"]:     # add the K4-shape fixture alone (the others are unchanged)
        fixture_steps(md, "split_step_b14.npz", B=14, nsteps=1, seed=7, data_seed=17)
        return
    check_split_equals_full(md)
    fixture_steps(md, "split_step_b4.npz", B=4, nsteps=3, weights_at=(1,))
    fixture_steps(md, "split_step_b1.npz", B=1, nsteps=1, seed=3, data_seed=7)
    fixture_steps(md, "split_step_b12.npz", B=12, nsteps=1, seed=5, data_seed=11)  # SplitFed 3x4 concat
    fixture_steps(md, "split_step_b13.npz", B=13, nsteps=1, seed=6, data_seed=13)  # ragged batch
    # BASELINE config 4's shape: SplitFed 7 clients x 2 samples, concatenated (round 6)
    fixture_steps(md, "split_step_b14.npz", B=14, nsteps=1, seed=7, data_seed=17)

    def ties(x, s):  # all-constant images: every pooling window is a 4-way tie
        x = torch.zeros_like(x)
        x[1] = 1.5
        return x
    fixture_steps(md, "split_step_ties_b2.npz", B=2, nsteps=1, seed=1, data_seed=5, xform=ties)
    fixture_curve(md, "loss_curve_b64.npz", B=64, nsteps=1000)


if __name__ == "__main__":
    main()
