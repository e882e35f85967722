"""Experiment: the C2 training step with the backward's side-stream work (per-layer dW1e, slab
reductions, encoder-node backward) kept on the side stream (default) or queued on the launch stream
(`main`), to see whether the overlap pays at 2 workgroups per CU.

  python tools/exp_side_stream.py default|main      # on the GPU box; prints the bench line"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from sgnn_amd import training

if sys.argv[1] == "main":
    _side = training.TrainWorkspace.side

    def side(self, device):
        s, ev = _side(self, device)
        return torch.cuda.current_stream(device), ev
    training.TrainWorkspace.side = side
bench.main(["--mode", "train", "--workload", "c2", "--no-extras", "--cpu-steps", "0", "--steps", "20", "--warmup", "5"])
