"""The multi-GPU bench's collectives on RCCL, at world size 1 on the one GPU the
test box has: the process-group init bench.py's ranks use (`nccl` bound to the rank's device),
the setup broadcast, the batch gather of u0 and the MAX / SUM aggregation, each from
rmpc.workloads exactly as bench.py calls them.  World size 2 of the same functions runs on gloo
in tests/test_multirank_cpu.py; RCCL at N > 1 needs the driver's multi-GPU node."""
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_world1_bench_collectives(gpu_lib, tmp_path):
    import torch
    import torch.distributed as dist
    from rmpc import workloads as W

    dev = torch.device("cuda:0")
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
        obs = torch.tensor([[2.0, 0.0, 0.4], [-1.5, 0.5, 0.3]], dtype=torch.float64, device=dev)
        ref = obs.clone()
        assert W.broadcast_shared(dist, obs) is obs and torch.equal(obs, ref)
        u0 = torch.randn(4096, 2, dtype=torch.float64, device=dev)
        g, out = W.gather_interleaved(dist, u0, 1)
        assert g.shape == (4096, 2) and torch.equal(g, u0)
        g2, out2 = W.gather_interleaved(dist, u0 * 2, 1, out)        # the reused output buffer
        assert out2 is out and torch.equal(g2, u0 * 2)
        el, counts = W.aggregate(dist, 1.25, [65530, 4, 2], device=dev)
        assert el == 1.25 and counts == [65530, 4, 2]
        dist.barrier()
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
