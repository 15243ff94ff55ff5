"""FedAvg round on the GPU stages over RCCL. With one rank the round is the
reference's single-client federated epoch (client_part.py:143-195 + the identity load_state_dict of
server_part.py:81): local full-model steps, then the state comes back unchanged. The B=4 fixture's
three split steps are exactly such a local epoch, so its post-step weights pin the result."""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import load_fixture, weight_ok


@pytest.mark.gpu
def test_fedavg_single_rank_rccl_matches_fixture(gpu):
    import torch.distributed as dist
    from splitcnn import dist as sd
    from splitcnn.data import init_models
    from splitcnn.engine import ClientStage, LossLog, ServerStage

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu)
    try:
        fx = load_fixture("split_step_b4.npz")
        a, b = init_models(seed=0)
        fed = sd.FedAvg(ClientStage(a, device=gpu), ServerStage(b, device=gpu, loss_log=LossLog(gpu)))
        n = int(fx["nsteps"])
        for k in range(1, n + 1):
            fed.local_step(torch.from_numpy(fx[f"x_{k}"]).to(gpu), torch.from_numpy(fx[f"y_{k}"]).to(gpu))
        fed.aggregate(step=n - 1)
        torch.cuda.synchronize()
        got = {"W1": a.conv1.weight, "b1": a.conv1.bias, "W2": b.conv2.weight, "b2": b.conv2.bias,
               "W3": b.fc1.weight, "b3": b.fc1.bias}
        for key, v in got.items():
            assert weight_ok(v.detach().cpu().numpy(), fx[f"post_{key}_{n}"], fx[f"init_{key}"]), key
        (step, loss), = fed.server.loss_log.flush()
        want = np.mean([float(fx[f"loss_{k}"]) for k in range(1, n + 1)])
        assert step == n - 1 and abs(loss - want) <= 1e-5 * want
    finally:
        dist.destroy_process_group()
