"""Drop-in for the reference package `checkpoint_utils` (src/checkpoint_utils/__init__.py:1-2).

Host-side checkpoint and metrics I/O used by train/train_BoostedNeuralLDPCDecoder.py (out of the
decode path's scope; kept so the reference's harness runs unchanged)."""
from checkpoint_utils.CheckPointUtil import CheckPointUtil
from checkpoint_utils.MetricsLogger import MetricsLogger

__all__ = ["CheckPointUtil", "MetricsLogger"]
