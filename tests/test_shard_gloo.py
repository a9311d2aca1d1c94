"""Frame sharding on CPU: shard ranges, and a world_size-2 gloo run of the sampler.

The per-frame function is the CPU oracle on the tiny UNet config (the HIP path needs a GPU); what is
under test is the sharding/timing host logic that bench.py and the multi-GPU run use: every frame is
processed exactly once, results equal the unsharded run, and only the timing is reduced.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from depth_completion_amd.shard import frame_shard, max_over_ranks, run_shard


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 2), (8, 8), (13, 4), (3, 8), (64, 8)])
def test_frame_shard_partition(n, world):
    ranges = [frame_shard(n, r, world) for r in range(world)]
    flat = [i for r in ranges for i in r]
    assert flat == list(range(n))  # contiguous, ordered, each frame exactly once
    sizes = [len(r) for r in ranges]
    assert max(sizes) - min(sizes) <= 1


def test_frame_shard_errors():
    with pytest.raises(ValueError):
        frame_shard(4, 2, 2)
    with pytest.raises(ValueError):
        frame_shard(4, 0, 0)


def _frames(n):
    g = torch.Generator().manual_seed(3)
    out = []
    for i in range(n):
        img = torch.randint(0, 256, (3, 32, 48), generator=g, dtype=torch.uint8)
        sp = torch.where(torch.rand((1, 32, 48), generator=g) < 0.05, 5 + 50 * torch.rand((1, 32, 48), generator=g),
                         torch.zeros(()))
        out.append((img, sp))
    return out


def _sampler():
    from oracle import pipeline_ref as P
    from oracle.diffusers_ref import (AutoencoderTiny, DDIMScheduler, UNet2DConditionModel, synthetic_state_dict,
                                      synthetic_taesd_state_dict, synthetic_text_embedding, tiny_unet_config)
    torch.set_num_threads(1)
    cfg = tiny_unet_config()
    unet = UNet2DConditionModel(cfg)
    unet.load_state_dict(synthetic_state_dict(unet, 11))
    vae = AutoencoderTiny()
    vae.load_state_dict(synthetic_taesd_state_dict(vae, 12))
    pipe = P.OracleMarigoldDC(unet, vae, DDIMScheduler(), synthetic_text_embedding(13, cfg.cross_attention_dim))

    def fn(frames, prev):
        imgs = torch.stack([f[0] for f in frames])
        sps = torch.stack([f[1] for f in frames])
        return pipe(imgs, sps, 60.0, norm="const", steps=2, resolution=48, pred_latents_prev=prev)
    return fn


def _worker(rank, world, port, n, use_prev, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        outs, el = run_shard(_sampler(), _frames(n), rank, world, use_prev_latent=use_prev)
        t = max_over_ranks(el)
        q.put((rank, [(i, d.float().numpy(), l.float().numpy()) for i, d, l in outs], el, t))  # by value
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("use_prev", [False, True])
def test_gloo_two_rank_sharding_matches_single(use_prev):
    n, world = 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, use_prev, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    got = {i: (torch.from_numpy(d), torch.from_numpy(l)) for _, outs, _, _ in res for i, d, l in outs}
    assert sorted(got) == list(range(n))
    tmax = max(r[2] for r in res)
    assert all(abs(r[3] - tmax) < 1e-9 for r in res)  # every rank sees the max-over-ranks time

    # single-process reference: the same shards' chains (the warm start restarts at the seam)
    fn = _sampler()
    frames = _frames(n)
    for r in range(world):
        ref, _ = run_shard(fn, frames, r, world, use_prev_latent=use_prev)
        for i, d, lat in ref:
            torch.testing.assert_close(got[i][0], d.float(), rtol=0, atol=0)
            torch.testing.assert_close(got[i][1], lat.float(), rtol=0, atol=0)
    if use_prev:  # the unsharded chain differs from the sharded one only after the seam
        full, _ = run_shard(fn, frames, 0, 1, use_prev_latent=True)
        torch.testing.assert_close(got[0][0], full[0][1].float(), rtol=0, atol=0)
