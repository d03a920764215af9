"""Trainer scalar logging with the reference's ML-Agents tag names.

The reference writes TensorBoard event files (``SummaryWriter``,
poca_trainer.py:358-360, 946-1033; option_critic_trainer.py:839-873;
learned_option_critic_trainer.py:1913-2141). When ``torch.utils.tensorboard``
is importable the same writer is used; otherwise (this image has no
tensorboard) every ``add_scalar`` / ``add_text`` call is appended as one JSON
line to ``<log_dir>/scalars.jsonl`` — same tags, values and steps, readable
with pandas (``pd.read_json(path, lines=True)``).
"""

from __future__ import annotations

import json
import os
import time


class JsonlScalarWriter:
    """SummaryWriter-compatible subset: add_scalar, add_text, flush, close."""

    def __init__(self, log_dir: str):
        self.log_dir = str(log_dir)
        os.makedirs(self.log_dir, exist_ok=True)
        self.path = os.path.join(self.log_dir, "scalars.jsonl")
        self._f = open(self.path, "a", buffering=1)

    def add_scalar(self, tag: str, value, step: int):
        self._f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step),
                                  "wall_time": time.time()}) + "\n")

    def add_text(self, tag: str, text: str, step: int = 0):
        self._f.write(json.dumps({"tag": tag, "text": str(text), "step": int(step), "wall_time": time.time()}) + "\n")

    def flush(self):
        self._f.flush()

    def close(self):
        if not self._f.closed:
            self._f.close()


class NullWriter:
    """Writer of the non-zero ranks of a multi-GPU run (rank 0 logs)."""

    def add_scalar(self, *a, **k):
        pass

    def add_text(self, *a, **k):
        pass

    def flush(self):
        pass

    def close(self):
        pass


def make_writer(log_dir: str, rank: int = 0):
    if rank != 0:
        return NullWriter()
    try:
        from torch.utils.tensorboard import SummaryWriter  # noqa: PLC0415
    except Exception:   # tensorboard not installed
        return JsonlScalarWriter(log_dir)
    return SummaryWriter(log_dir=log_dir)


def read_scalars(log_dir: str) -> list[dict]:
    with open(os.path.join(log_dir, "scalars.jsonl")) as f:
        return [json.loads(line) for line in f if line.strip()]
