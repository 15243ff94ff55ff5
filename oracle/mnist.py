"""ORACLE — TEST INFRASTRUCTURE ONLY. Never imported by the product path (splitcnn/).

The reference's input transform, restated in numpy float32: torchvision 0.17.0 (pinned in
src/requirements.txt:3; not installed here) as configured at src/client_part.py:61-64:
  ToTensor:   u8 image -> float32, .div(255)            (transforms.functional.to_tensor)
  Normalize:  .sub_(mean).div_(std), mean/std float32    (transforms.functional.normalize)
and the batch gather of DataLoader(batch_size=64, shuffle=True) (client_part.py:98) for a given
index order. torchvision is absent, so the pin is the torch CPU op sequence those two functions run
(tests/test_mnist.py::test_oracle_equals_torch_op_sequence), bit for bit.
"""
import numpy as np

MEAN = np.float32(0.1307)
STD = np.float32(0.3081)


def transform(images_u8: np.ndarray) -> np.ndarray:
    """u8 [..., 28, 28] -> f32 [..., 1, 28, 28] exactly as ToTensor + Normalize."""
    t = images_u8.astype(np.float32) / np.float32(255.0)
    t = (t - MEAN) / STD
    return t.reshape(t.shape[:-2] + (1,) + t.shape[-2:]).astype(np.float32)


def batch(images_u8: np.ndarray, labels_u8: np.ndarray, idx: np.ndarray):
    """(x f32 [B,1,28,28], y i64 [B]) for the rows `idx` (one DataLoader batch)."""
    return transform(images_u8[idx]), labels_u8[idx].astype(np.int64)
