"""splitcnn — MI355X-native split-learning engine for the split-CNN step of
eliasandronicou/split-learning-k8s.

Module contract (drop-in for src/model_def.py): ModelPartA, ModelPartB, FullModel, get_model.
Step contract (src/client_part.py <-> src/server_part.py): ClientStage, ServerStage, SplitTrainer.
"""
from .model_def import (CrossEntropyLoss, FullModel, ModelPartA, ModelPartB,  # noqa: F401
                        get_model)

__all__ = ["ModelPartA", "ModelPartB", "FullModel", "get_model", "CrossEntropyLoss"]


def __getattr__(name):
    # engine pieces are imported lazily so `import splitcnn` stays light
    if name in ("ClientStage", "ServerStage", "SplitTrainer", "LossLog"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
