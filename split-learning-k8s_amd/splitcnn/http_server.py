"""HTTP-compatible server adapter: the reference's FastAPI server contract
(src/server_part.py:1-102) backed by the MI355X ServerStage.

Wire format is the reference's: POST /forward_pass with a pickled
{"activations": f32[B,32,26,26], "labels": i64[B], "step": int} (src/client_part.py:117-125) returns
the pickled cut gradient (src/server_part.py:57-58) or 400 with a text body when LEARNING_MODE is not
"split" (server_part.py:32-36). POST /aggregate_weights implements the federated endpoint
(server_part.py:60-93): with `fed_clients=1` it returns the received state (the reference's
identity "aggregation"); with K clients each request waits for the round's K states and gets
their mean (FedAvg with equal weights: the reference payload carries no sample count). GET /health mirrors server_part.py:95-102. So the unmodified reference client
(src/client_part.py) can train against it by pointing SERVER_URL_SPLIT here.

Differences by design:
  - request bodies are unpickled with an allow-list (torch tensor rebuild + plain containers), not
    bare pickle.loads: the reference executes whatever a POST body says;
  - the loss is logged to the device LossLog (flushed every `flush_every` steps to `sink`), not a
    blocking MLflow REST call per request (server_part.py:55);
  - a lock keeps requests serialised against the one server model, like the reference's single
    uvicorn worker; the ServerStage (and the GPU) is created on the first /forward_pass.
"""

import asyncio
import io
import logging
import os
import pickle
import threading
from typing import Callable, Optional

import torch

_ALLOWED = {
    ("torch._utils", "_rebuild_tensor_v2"), ("torch._utils", "_rebuild_tensor"),
    ("torch._utils", "_rebuild_parameter"), ("collections", "OrderedDict"), ("torch", "Size"),
}


def _load_storage_bytes(b: bytes):
    # torch pickles a tensor's storage as torch.storage._load_from_bytes(<torch.save bytes>), which
    # would run torch.load(weights_only=False); the weights-only loader accepts exactly storages.
    return torch.load(io.BytesIO(b), weights_only=True)


class SafeUnpickler(pickle.Unpickler):
    """Unpickle only tensors and plain containers (what the reference client sends)."""

    def find_class(self, module, name):
        if (module, name) == ("torch.storage", "_load_from_bytes"):
            return _load_storage_bytes
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refused to unpickle {module}.{name}")

    def persistent_load(self, pid):  # pickle.dumps never emits these; torch.save archives are refused
        raise pickle.UnpicklingError("persistent ids are not accepted")


def safe_loads(data: bytes):
    return SafeUnpickler(io.BytesIO(data)).load()


log = logging.getLogger("splitcnn.http")


def make_app(server=None, device: str = "cuda", learning_mode: Optional[str] = None,
             sink: Optional[Callable[[int, float], None]] = None, flush_every: int = 100,
             fed_clients: int = 1, fed_timeout: float = 600.0):
    """Build the FastAPI app. `server` defaults to a seeded ServerStage on `device`.

    Federated rounds (fed_clients = K > 1): a round closes when K states have arrived. A request may
    carry an optional "client_id"; a second post from the same id in an open round is refused (409)
    instead of being counted twice. A round that does not fill within `fed_timeout` seconds is
    abandoned: every waiting client gets 504 and the next post opens a fresh round."""
    from fastapi import FastAPI, Request, Response

    from .engine import LossLog, ServerStage
    from .model_def import FullModel, get_model

    mode = (learning_mode or os.getenv("LEARNING_MODE", "split")).lower()
    app = FastAPI()
    lock = threading.Lock()
    state = {"server": server, "full": None, "since_flush": 0}

    def split_server():
        if state["server"] is None:
            state["server"] = ServerStage(get_model(role="server"), device=device,
                                          loss_log=LossLog(device, sink=sink))
        return state["server"]

    @app.post("/forward_pass")
    async def forward_pass(request: Request):
        if mode != "split":
            return Response(content=f"Error: /forward_pass endpoint is only for split learning mode. "
                                    f"Current mode: {mode}", status_code=400)
        body = await request.body()
        try:
            data = safe_loads(body)
            act = data["activations"]
            labels = data["labels"]
            step = int(data["step"])
            if tuple(act.shape[1:]) != (32, 26, 26) or labels.shape != (act.shape[0],):
                raise ValueError(f"activations {tuple(act.shape)} / labels {tuple(labels.shape)}")
        except Exception as e:  # malformed / refused payload
            return Response(content=f"Error: bad payload ({e})", status_code=400)
        if labels.numel() and (int(labels.min()) < 0 or int(labels.max()) >= 10):
            # the reference's criterion raises IndexError before its SGD step (server_part.py:50)
            return Response(content="Error: Target out of bounds (labels must be in [0, 10))",
                            status_code=500)
        with lock:
            s = split_server()
            act = act.to(s.device, dtype=torch.float32).contiguous()
            labels = labels.to(s.device, dtype=torch.int64).contiguous()
            cut_grad, _ = s.step_request(act, labels, step=step)
            out = cut_grad.detach().cpu()
            state["since_flush"] += 1
            if state["since_flush"] >= flush_every:
                state["since_flush"] = 0
                try:
                    s.loss_log.flush()
                except Exception as e:  # the step is applied: a sink outage must not turn it into a 500
                    log.warning("loss sink flush failed (metrics stay buffered in the sink): %r", e)
        return Response(content=pickle.dumps(out), media_type="application/octet-stream")

    fed = {"round": None}

    @app.post("/aggregate_weights")
    async def aggregate_weights(request: Request):
        if mode != "federated":
            return Response(content=f"Error: /aggregate_weights endpoint is only for federated learning mode. "
                                    f"Current mode: {mode}", status_code=400)
        try:
            data = safe_loads(await request.body())
            client_state = data["model_state"]
            epoch, client_loss, step = data["epoch"], data["loss"], data["step"]
            client_id = data.get("client_id")
        except Exception as e:
            return Response(content=f"Error: bad payload ({e})", status_code=400)
        # A round closes when `fed_clients` states have arrived; every waiting client gets the mean.
        # fed_clients=1 is the reference's identity aggregation (server_part.py:81).
        rnd = fed["round"]
        if rnd is None:
            rnd = fed["round"] = {"states": [], "losses": [], "ids": set(), "done": asyncio.Event(),
                                  "out": None, "error": None}
        if client_id is not None:
            if client_id in rnd["ids"]:
                return Response(content=f"Error: client {client_id!r} already posted to this round",
                                status_code=409)
            rnd["ids"].add(client_id)
        rnd["states"].append(client_state)
        rnd["losses"].append((int(step), float(client_loss), float(epoch)))
        if len(rnd["states"]) >= fed_clients:
            fed["round"] = None
            try:
                with lock:
                    if state["full"] is None:
                        state["full"] = FullModel()
                    m = state["full"]
                    avg = {k: torch.stack([sd[k].float() for sd in rnd["states"]]).mean(0)
                           for k in rnd["states"][0]}
                    m.load_state_dict(avg)
                    if sink is not None:
                        # mlflow.log_metric("loss" / "epoch", ..., step=step)  (server_part.py:86-87)
                        st = max(s for s, _, _ in rnd["losses"])
                        mean_loss = sum(l for _, l, _ in rnd["losses"]) / len(rnd["losses"])
                        try:
                            if hasattr(sink, "log_metric"):
                                sink.log_metric("loss", mean_loss, st)
                                sink.log_metric("epoch", max(e for _, _, e in rnd["losses"]), st)
                            else:
                                sink(st, mean_loss)
                            if hasattr(sink, "flush"):
                                sink.flush()
                        except Exception as e:
                            log.warning("metric sink failed (metrics stay buffered in the sink): %r", e)
                    rnd["out"] = pickle.dumps(m.state_dict())
            except Exception as e:  # every waiter of this round gets the 500 now, not at its timeout
                rnd["error"] = (500, f"Error: federated aggregation failed ({e!r})")
            finally:
                rnd["done"].set()
        else:
            try:
                await asyncio.wait_for(rnd["done"].wait(), timeout=fed_timeout)
            except asyncio.TimeoutError:
                if fed["round"] is rnd:
                    fed["round"] = None   # abandon the partial round: release every other waiter at once
                    rnd["error"] = (504, f"Error: federated round incomplete after {fed_timeout}s "
                                         f"({len(rnd['states'])}/{fed_clients} clients)")
                    rnd["done"].set()
                if rnd["error"] is None:  # completed concurrently with the timeout
                    return Response(content=rnd["out"], media_type="application/octet-stream")
        if rnd["error"] is not None:
            return Response(content=rnd["error"][1], status_code=rnd["error"][0])
        return Response(content=rnd["out"], media_type="application/octet-stream")

    @app.get("/health")
    async def health():
        return {"status": "healthy", "mode": mode,
                "model_type": "FullModel" if mode == "federated" else "ModelPartB"}

    @app.get("/losses")
    async def losses():
        """Flushed (step, loss) pairs — the local stand-in for the MLflow metric view."""
        with lock:
            s = state["server"]
            if s is None:
                return {"losses": []}
            s.loss_log.flush()
            return {"losses": s.loss_log.history}

    return app

