"""One rank of tests/test_gpu_dp.py: a fresh process that joins a gloo group
(several ranks share the one leased GPU; RCCL refuses two ranks on one
device) or, for the RCCL cases, a one-rank nccl group, runs its share of the global batch through the HIP trainer and saves
loss, gradient and parameters.  Usage: gpu_dp_child.py CASE RANK WORLD PORT OUT"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    case, rank, world, port, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    import torch
    import torch.distributed as dist
    from tests.dp_cases import CASES, MS_CASES, RCCL_CASES
    if case in RCCL_CASES:   # RCCL (backend "nccl" on ROCm), one rank on the one GPU
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    run, _, ranks = CASES[case]
    res = run(ranks[rank], global_ids=sum(ranks, [])) if case in MS_CASES else run(ranks[rank])
    torch.save(res, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
