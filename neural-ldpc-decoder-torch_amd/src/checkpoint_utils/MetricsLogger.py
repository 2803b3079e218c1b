"""Text metrics log (reference: src/checkpoint_utils/MetricsLogger.py:5-71).

One line per logged epoch: `epoch, timestamp, metric values..., checkpoint file`; BER-like keys in
scientific notation.  A header with the config is written when epoch 0 is logged."""
import os
from datetime import datetime
from typing import Any, Dict, Optional


class MetricsLogger:
    def __init__(self, log_dir: str = "checkpoints", filename: str = "training_metrics.txt"):
        self.log_dir = log_dir
        self.log_file = os.path.join(log_dir, filename)
        os.makedirs(log_dir, exist_ok=True)
        self.best_ber = float("inf")

    def log(self, epoch: int, metrics: Dict[str, float], checkpoint_filename: str,
            config: Optional[Dict[str, Any]] = None):
        now = datetime.now().strftime("%Y-%m-%d %H:%M:%S")
        if epoch == 0 and config is not None:
            with open(self.log_file, "w") as f:
                f.write(f"# Training started: {now}\n")
                f.write("# Config: " + ", ".join(f"{k}={v}" for k, v in config.items()) + "\n")
                f.write("# Columns: Epoch, Timestamp, " + ", ".join(metrics.keys()) + ", Checkpoint_File\n")
                f.write("-" * 120 + "\n")
        vals = [f"{v:.6e}" if "ber" in k.lower() else f"{v:.6f}" for k, v in metrics.items()]
        with open(self.log_file, "a") as f:
            f.write(f"{epoch:4d}, {now}, " + ", ".join(vals) + f", {checkpoint_filename}\n")

    def is_best(self, ber: float) -> bool:
        if ber < self.best_ber:
            self.best_ber = ber
            return True
        return False
