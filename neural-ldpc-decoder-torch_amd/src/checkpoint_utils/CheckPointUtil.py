"""Checkpoint save / load (reference: src/checkpoint_utils/CheckPointUtil.py:8-159).

save(): {'model_state_dict', 'optimizer_state_dict'?, 'epoch'?, **metrics, 'config'?} via torch.save.
save_weights(): state_dict as .pth, optionally one numpy text file per entry plus an index.
load(): torch.load with weights_only=True (no pickled code is executed), then load_state_dict.
"""
import os
from datetime import datetime
from typing import Any, Dict, Optional

import numpy as np
import torch


class CheckPointUtil:
    def __init__(self, checkpoint_dir: str = "checkpoints"):
        self.checkpoint_dir = checkpoint_dir
        os.makedirs(checkpoint_dir, exist_ok=True)

    def _path(self, filepath: str) -> str:
        return filepath if os.path.isabs(filepath) else os.path.join(self.checkpoint_dir, filepath)

    def save(self, filepath: str, model: torch.nn.Module, optimizer: Optional[torch.optim.Optimizer] = None,
             epoch: Optional[int] = None, metrics: Optional[Dict[str, float]] = None,
             config: Optional[Dict[str, Any]] = None) -> str:
        data: Dict[str, Any] = {"model_state_dict": model.state_dict()}
        if optimizer is not None:
            data["optimizer_state_dict"] = optimizer.state_dict()
        if epoch is not None:
            data["epoch"] = epoch
        if metrics is not None:
            data.update(metrics)
        if config is not None:
            data["config"] = config
        path = os.path.join(self.checkpoint_dir, filepath)
        torch.save(data, path)
        return path

    def save_weights(self, filepath: str, model: torch.nn.Module, as_txt: bool = False) -> str:
        pth = filepath if filepath.endswith(".pth") else filepath + ".pth"
        path = os.path.join(self.checkpoint_dir, pth)
        state = model.state_dict()
        torch.save(state, path)
        if as_txt:
            txt_dir = os.path.join(self.checkpoint_dir, f"{filepath.replace('.pth', '')}_weights_txt")
            os.makedirs(txt_dir, exist_ok=True)
            lines = [f"# Model weights saved at: {datetime.now().strftime('%Y-%m-%d %H:%M:%S')}",
                     f"# Total parameters: {sum(p.numel() for p in model.parameters())}",
                     "# Format: Each parameter saved in separate .txt file", "-" * 80,
                     "Parameter_Name, Shape, Filename"]
            for name, value in state.items():
                fname = name.replace(".", "_").replace("/", "_") + ".txt"
                arr = value.detach().cpu().numpy()
                if arr.ndim > 2:
                    np.savetxt(os.path.join(txt_dir, fname), arr.reshape(arr.shape[0], -1),
                               header=f"Original shape: {arr.shape}\nReshaped to 2D for savetxt")
                else:
                    np.savetxt(os.path.join(txt_dir, fname), arr)
                lines.append(f"{name}, {list(value.shape)}, {fname}")
            with open(os.path.join(txt_dir, "index.txt"), "w") as f:
                f.write("\n".join(lines) + "\n")
        return path

    def load(self, filepath: str, model: torch.nn.Module, optimizer: Optional[torch.optim.Optimizer] = None,
             device: Optional[torch.device] = None) -> Dict[str, Any]:
        ckpt = torch.load(self._path(filepath), map_location=device, weights_only=True)
        model.load_state_dict(ckpt["model_state_dict"])
        if optimizer is not None and "optimizer_state_dict" in ckpt:
            optimizer.load_state_dict(ckpt["optimizer_state_dict"])
        return ckpt
