"""Checkpoint / resume (utils/checkpoint_utils.py:5-42, train.py:364-391).

Files are interchangeable with the reference's: the model file is the
simulator's `state_dict()` (same keys), the train-state file is
`{"optimizer_state": torch.optim.Adam.state_dict(), "global_train_state":
{"step": ..., ...}}`.  Loading never unpickles code (`weights_only=True`).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch


def save_train_state(path: str, optimizer_state: dict, step: int, **extra) -> None:
    """train.py:369-374 / :403-407."""
    torch.save({"optimizer_state": optimizer_state, "global_train_state": dict(step=step, **extra)}, path)


def load_train_state(path: str) -> dict:
    return torch.load(path, map_location="cpu", weights_only=True)


def load_model(simulator: torch.nn.Module, model_dir: str, model_file: str, train_state_file: str,
               device, trainer=None) -> Tuple[torch.nn.Module, int, dict]:
    """checkpoint_utils.py:13-42: weights + optimizer state + step.

    With `trainer` (a sgnn_amd.train.Trainer built on `simulator`) the
    optimizer moments, step count and LR are loaded into its fused Adam and the
    trainer continues at the saved step (the reference resets `step` to 0 after
    resuming, train.py:225 — SURVEY Appendix A.18 — which is not reproduced).
    Returns (simulator, step, optimizer_state_dict)."""
    model_path = model_dir + model_file
    state_path = model_dir + train_state_file
    if not (os.path.exists(model_path) and os.path.exists(state_path)):
        raise FileNotFoundError(f"Specified model_file {model_path} and train_state_file {state_path} not found.")
    simulator.load(model_path)
    simulator.to(device)
    ts = load_train_state(state_path)
    step = int(ts["global_train_state"]["step"])
    if trainer is not None:
        trainer.opt.load_state_dict(ts["optimizer_state"])
        trainer.step = step
    return simulator, step, ts["optimizer_state"]
