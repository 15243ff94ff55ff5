"""Loss sinks for LossLog: where the reference calls mlflow.log_metric("loss", loss,
step=step) once per request (src/server_part.py:55, tracking server at server_part.py:19-24), the
device loss log is flushed every N steps and hands its (step, loss) pairs to a sink.

MlflowRestSink speaks the MLflow tracking REST API directly (the `mlflow` package is not needed):
it gets-or-creates the experiment "<Mode>_Learning_Sim" and a run "<Mode>_Training" like
server_part.py:20-24, buffers metrics, and posts them with runs/log-batch (≤1000 per request) when
the LossLog flushes. JsonlSink appends one JSON object per metric to a local file.
"""
import json
import time
from typing import List, Optional


class JsonlSink:
    def __init__(self, path: str, key: str = "loss"):
        self.path, self.key = path, key
        self._pending: List[dict] = []

    def log_metric(self, key: str, value: float, step: int):
        """mlflow.log_metric(key, value, step=step) (server_part.py:55,86-87), buffered until flush."""
        self._pending.append({"key": key, "value": float(value), "step": int(step),
                              "timestamp": int(time.time() * 1000)})

    def __call__(self, step: int, value: float):
        self.log_metric(self.key, value, step)

    def flush(self):
        if self._pending:
            with open(self.path, "a") as f:
                for m in self._pending:
                    f.write(json.dumps(m) + "\n")
            self._pending.clear()


class MlflowRestSink:
    BATCH = 1000  # MLflow's log-batch metric limit

    def __init__(self, tracking_uri: str, mode: str = "split", run_id: Optional[str] = None,
                 key: str = "loss", timeout: float = 10.0):
        import requests
        self._http = requests.Session()
        self.uri = tracking_uri.rstrip("/")
        self.key = key
        self.timeout = timeout
        self._pending: List[dict] = []
        self.run_id = run_id or self._start_run(mode)

    def _api(self, method: str, path: str, **kw):
        r = self._http.request(method, f"{self.uri}/api/2.0/mlflow/{path}", timeout=self.timeout, **kw)
        return r

    def _start_run(self, mode: str) -> str:
        name = f"{mode.capitalize()}_Learning_Sim"           # server_part.py:20
        r = self._api("GET", "experiments/get-by-name", params={"experiment_name": name})
        if r.status_code == 200:
            exp_id = r.json()["experiment"]["experiment_id"]
        else:
            r = self._api("POST", "experiments/create", json={"name": name})
            r.raise_for_status()
            exp_id = r.json()["experiment_id"]
        r = self._api("POST", "runs/create", json={"experiment_id": exp_id,
                                                   "run_name": f"{mode.capitalize()}_Training",  # :23
                                                   "start_time": int(time.time() * 1000)})
        r.raise_for_status()
        return r.json()["run"]["info"]["run_id"]

    def log_metric(self, key: str, value: float, step: int):
        self._pending.append({"key": key, "value": float(value), "step": int(step),
                              "timestamp": int(time.time() * 1000)})

    def __call__(self, step: int, value: float):
        self.log_metric(self.key, value, step)

    def flush(self):
        """Post the buffered metrics in log-batch chunks. A chunk leaves the buffer only after the
        tracking server accepted it, so a failed post (raised) is retried by the next flush."""
        while self._pending:
            chunk = self._pending[:self.BATCH]
            r = self._api("POST", "runs/log-batch", json={"run_id": self.run_id, "metrics": chunk})
            r.raise_for_status()
            del self._pending[:len(chunk)]
