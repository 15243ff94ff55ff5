"""`from model_def import get_model` shim: with split-learning-k8s_amd/ on sys.path (where the
reference puts src/), the reference's client/server code imports this module unchanged and gets the
MI355X-native modules (src/model_def.py:1-71 contract)."""
from splitcnn.model_def import (FullModel, ModelPartA, ModelPartB,  # noqa: F401
                                get_model)
