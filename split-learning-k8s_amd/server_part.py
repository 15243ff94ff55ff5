"""Drop-in for the reference's src/server_part.py: `uvicorn server_part:app` (k8s/split-learning.yaml:34)
serves /forward_pass, /aggregate_weights and /health with the MI355X server stage behind them
(splitcnn/http_server.py)."""
from splitcnn.http_server import make_app

app = make_app()
