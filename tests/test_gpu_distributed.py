"""BASELINE configs[3]'s data-parallel step with the real engine in every rank:
two spawned processes (world 2, gloo, both on the box's one GPU) each run
ResNet18Int8.forward through libdlq.so on their shard of the batch inside
bench.GatherPipeline (async all-gather of the logits, two slots), and the
gathered logits equal a single process's forward over the whole batch, bit
for bit.  The logits are gathered through host tensors (gloo); on the 8-GPU
node bench.py runs the same pipeline over RCCL on device tensors.

Per-rank batch 256 = the real configs[3] shard (B = 2048 over 8 ranks)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, per, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from dlq_amd.models import ResNet18Int8, synthetic_images
        from dlq_amd.lib import lib
        from tests.helpers import model_and_scales
        torch.cuda.set_device(0)
        sd, scales = model_and_scales()
        x_all = synthetic_images(per * world, seed=31)
        x_local = x_all[rank * per:(rank + 1) * per].cuda().contiguous()
        model = ResNet18Int8(sd, scales, max_batch=per)
        dev_logits = torch.empty((per, 1000), dtype=torch.float32, device="cuda")

        def fwd_into(x, out):  # the engine on this rank's GPU, logits to the host slot
            model.forward(x, dev_logits)
            out.copy_(dev_logits.cpu())

        pipe = bench.GatherPipeline(fwd_into, per, world, "cpu")
        flip = torch.flip(x_local, dims=[0]).contiguous()
        k1 = pipe.step(x_local)
        k2 = pipe.step(flip)
        pipe.finish()
        p1, p2 = pipe.out[k1].clone(), pipe.out[k2].clone()
        k3 = pipe.step(x_local)  # reuses slot k1 after its gather was waited on
        pipe.finish()
        loaded = any("libdlq.so" in l for l in open("/proc/self/maps"))
        if rank == 0:
            q.put((p1.numpy(), p2.numpy(), pipe.out[k3].numpy(), (k1, k2, k3), loaded))
        else:
            q.put(("rank1", loaded))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("per", [3, 256])
def test_dp_world2_engine_gather(gpu, per):
    from dlq_amd.models import ResNet18Int8, synthetic_images
    from tests.helpers import model_and_scales
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0 = next(r for r in res if not isinstance(r[0], str))
    r1 = next(r for r in res if isinstance(r[0], str))
    p1, p2, p3, slots, loaded0 = r0
    assert loaded0 and r1[1], "both ranks must run libdlq.so"
    # one process, the whole batch
    sd, scales = model_and_scales()
    x_all = synthetic_images(per * world, seed=31).cuda()
    ref = ResNet18Int8(sd, scales, max_batch=per * world)(x_all).cpu().numpy()
    assert slots == (0, 1, 0)
    assert p1.shape == (per * world, 1000)
    assert np.array_equal(p1.view(np.int32), ref.view(np.int32))
    ref_flip = np.concatenate([ref[r * per:(r + 1) * per][::-1] for r in range(world)])
    assert np.array_equal(p2.view(np.int32), ref_flip.view(np.int32))
    assert np.array_equal(p3.view(np.int32), ref.view(np.int32))
    if per <= 4:  # and the single process is the oracle's
        from oracle import oracle as O
        want, _ = O.resnet18_forward_s8(sd, scales, x_all.cpu().numpy())
        assert np.array_equal(ref.view(np.int32), want.view(np.int32))


def _worker8(rank, world, port, per, sd, scales, q):
    """One rank of BASELINE configs[3] on the box's one GPU: its own 256-image
    shard (seed 4000 + rank), the engine through bench.GatherPipeline."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from dlq_amd.models import ResNet18Int8, synthetic_images
        torch.cuda.set_device(0)
        x_local = synthetic_images(per, seed=4000 + rank).cuda().contiguous()
        model = ResNet18Int8(sd, scales, max_batch=per)
        dev_logits = torch.empty((per, 1000), dtype=torch.float32, device="cuda")

        def fwd_into(x, out):
            model.forward(x, dev_logits)
            out.copy_(dev_logits.cpu())

        pipe = bench.GatherPipeline(fwd_into, per, world, "cpu")
        k = pipe.step(x_local)
        pipe.finish()
        loaded = any("libdlq.so" in l for l in open("/proc/self/maps"))
        q.put((rank, pipe.out[k].numpy() if rank == 0 else None, loaded))
    finally:
        dist.destroy_process_group()


def test_dp_world8_configs3_global_batch(gpu):
    """BASELINE configs[3] at its workload: world 8 x 256 images = 2048
    (gloo on the one GPU box; bench.py runs the same pipeline over RCCL on the
    8-GPU node).  The gathered [2048, 1000] logits equal one process's B = 2048
    forward bit for bit (anchor: the logits of infer_e2e.cu:206-219's fc_forward)."""
    from dlq_amd.models import ResNet18Int8, synthetic_images
    from tests.helpers import model_and_scales
    world, per = 8, 256
    sd, scales = model_and_scales()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker8, args=(r, world, port, per, sd, scales, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=400) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[2] for r in res), "every rank must run libdlq.so"
    got = next(r[1] for r in res if r[0] == 0)
    assert got.shape == (world * per, 1000)
    x_all = torch.cat([synthetic_images(per, seed=4000 + r) for r in range(world)]).cuda()
    ref = ResNet18Int8(sd, scales, max_batch=world * per)(x_all).cpu().numpy()
    assert np.array_equal(got.view(np.int32), ref.view(np.int32))


def _worker_rccl(port, per, sd, scales, q):
    """One rank over RCCL on the box's GPU: the nccl process group bound to
    cuda:0, the engine's logits gathered by all_gather_into_tensor on device
    tensors inside bench.GatherPipeline (the collective bench.py issues per
    step on the 8-GPU node, here with one rank)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import bench
        from dlq_amd.models import ResNet18Int8, synthetic_images
        x = synthetic_images(per, seed=77).cuda().contiguous()
        model = ResNet18Int8(sd, scales, max_batch=per)
        pipe = bench.GatherPipeline(lambda xx, out: model.forward(xx, out), per, 1, "cuda", exchange=True)
        flip = torch.flip(x, dims=[0]).contiguous()
        k1 = pipe.step(x)
        k2 = pipe.step(flip)
        pipe.finish()
        p1, p2 = pipe.out[k1].cpu(), pipe.out[k2].cpu()
        k3 = pipe.step(x)
        pipe.finish()
        torch.cuda.synchronize()
        same_storage = pipe.out[k1].data_ptr() == pipe.logits[k1].data_ptr()
        q.put((dist.get_backend(), p1.numpy(), p2.numpy(), pipe.out[k3].cpu().numpy(), (k1, k2, k3), same_storage))
    finally:
        dist.destroy_process_group()


def test_rccl_one_rank_gather_pipeline(gpu):
    """RCCL on MI355X: communicator init and the pipeline's async
    all_gather_into_tensor on device logits (one rank; the box has one GPU,
    and RCCL refuses two ranks on one device).  The gathered logits are a
    separate buffer holding the engine's logits bit for bit."""
    from dlq_amd.models import ResNet18Int8, synthetic_images
    from tests.helpers import model_and_scales
    per = 64
    sd, scales = model_and_scales()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_rccl, args=(_free_port(), per, sd, scales, q))
    p.start()
    backend, p1, p2, p3, slots, same = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl" and slots == (0, 1, 0) and not same
    x = synthetic_images(per, seed=77).cuda()
    ref = ResNet18Int8(sd, scales, max_batch=per)(x).cpu().numpy()
    assert np.array_equal(p1.view(np.int32), ref.view(np.int32))
    assert np.array_equal(p2.view(np.int32), ref[::-1].view(np.int32))
    assert np.array_equal(p3.view(np.int32), ref.view(np.int32))
