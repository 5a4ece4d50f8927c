"""Multi-process plumbing of bench.py (one process per GPU, torch.distributed: RCCL on the GPU box, gloo on
CPU). The reconstruction path has no data-path collective in this round: each rank decodes its own
stream segment (replicas of the same segment in the bench, SURVEY.md 8(e) "temporal" sharding), so the
only collectives are the timing barrier and the max-over-ranks of the elapsed time."""
import os


class Ranks:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.device = "cpu"
        if self.world > 1:
            import torch
            import torch.distributed as dist
            backend = os.environ.get("VVCR_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
            if backend == "nccl":
                torch.cuda.set_device(int(os.environ.get("VVCR_DEVICE", self.local)))   # VVCR_DEVICE: one-GPU rehearsal
                self.device = "cuda"
            dist.init_process_group(backend)
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, x):
        """The job's elapsed time is the slowest rank's."""
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, x):
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


def job_throughput(units_per_rank, elapsed_max, ranks):
    """Whole-job rate: the units all ranks processed / the slowest rank's time (weak scaling)."""
    return ranks.sum_over_ranks(units_per_rank) / elapsed_max
