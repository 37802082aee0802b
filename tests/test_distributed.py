"""CPU, world_size 2 over gloo: the data-parallel step of bench.py (shard the
batch by rank, run the forward locally, all-gather the logits) returns the
same [B,1000] logits, in the same order, as one process over the whole batch.
The per-rank forward here is the CPU oracle (the GPU engine is per-rank
identical and is covered by tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from oracle import oracle as O
        from dlq_amd.models import synthetic_images
        from tests.helpers import model_and_scales
        sd, scales = model_and_scales()
        x_all = synthetic_images(2 * world, seed=31)
        per = x_all.shape[0] // world
        x_local = x_all[rank * per:(rank + 1) * per]

        def fwd(x):
            return torch.from_numpy(O.resnet18_forward_s8(sd, scales, x.numpy())[0])

        out = bench.shard_gather(fwd, x_local, world)
        # the overlapped pipeline of the timed loop: async gathers, two slots
        pipe = bench.GatherPipeline(lambda x, o: o.copy_(fwd(x)), per, world, "cpu")
        flip = torch.flip(x_local, dims=[0]).contiguous()
        k1 = pipe.step(x_local)
        k2 = pipe.step(flip)
        pipe.finish()
        p1, p2 = pipe.out[k1].clone(), pipe.out[k2].clone()
        k3 = pipe.step(x_local)  # reuses slot k1 after its gather was waited on
        pipe.finish()
        if rank == 0:
            q.put((out.numpy(), p1.numpy(), p2.numpy(), pipe.out[k3].numpy(), (k1, k2, k3)))
    finally:
        dist.destroy_process_group()


def test_shard_and_allgather_world2():
    from oracle import oracle as O
    from dlq_amd.models import synthetic_images
    from tests.helpers import model_and_scales
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, p1, p2, p3, slots = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sd, scales = model_and_scales()
    x_all = synthetic_images(2 * world, seed=31).numpy()
    ref, _ = O.resnet18_forward_s8(sd, scales, x_all)
    assert got.shape == (2 * world, 1000)
    assert np.array_equal(got.view(np.int32), ref.view(np.int32))
    # pipeline: step 2 ran each rank's images in reverse order
    per = 2
    ref_flip = np.concatenate([ref[r * per:(r + 1) * per][::-1] for r in range(world)])
    assert slots == (0, 1, 0)
    assert np.array_equal(p1.view(np.int32), ref.view(np.int32))
    assert np.array_equal(p2.view(np.int32), ref_flip.view(np.int32))
    assert np.array_equal(p3.view(np.int32), ref.view(np.int32))
