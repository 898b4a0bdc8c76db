"""Data-parallel gradient exchange (train_step.flat_allreduce_mean) on 2 and 4
gloo ranks: each rank differentiates the oracle on its share of the rays (whole
4x4 patches); after the flat all-reduce every rank holds the single-process
gradient of the full batch."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import REN_CFG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(R, seed):
    g = torch.Generator().manual_seed(seed)
    o = torch.tensor([0.05, -0.03, 1.6]).expand(R, 3).contiguous()
    d = torch.cat([(torch.rand(R, 2, generator=g) - 0.5) * 0.5, -torch.ones(R, 1)], -1)
    n = d.norm(dim=-1, keepdim=True)
    return o, d / n, n, torch.rand(R, 64, generator=g), torch.rand(R, 3, generator=g)


def _grads(rows):
    from helpers import build_modules, oracle_params
    from oracle import neus_oracle as O
    P, Pc, var, leaves = oracle_params(*build_modules(9, 64, 64))
    o, d, n, tr, gt = rows
    R = o.shape[0]
    out = O.render(P, Pc, var, o, d, n, torch.tensor([0.1]), torch.full((R, 1), 0.01), torch.full((R, 1), 3.0),
                   car=0.5, t_rand=tr, n_samples=REN_CFG["n_samples"], n_importance=REN_CFG["n_importance"])
    loss = O.train_loss(out, gt)
    names = list(leaves)
    gr = torch.autograd.grad(loss, [leaves[k] for k in names])
    return names, gr


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "cope-nerf_amd"), root, os.path.join(root, "tests")]
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from copenerf.train_step import flat_allreduce_mean
    full = _batch(16 * world, 0)
    part = tuple(t[rank * 16:(rank + 1) * 16] for t in full)  # one whole 4x4 patch group per rank
    names, gr = _grads(part)
    params = [torch.nn.Parameter(torch.zeros_like(g)) for g in gr]
    for p, g in zip(params, gr):
        p.grad = g.clone()
    flat_allreduce_mean(params)
    q.put((rank, {n: p.grad.numpy().copy() for n, p in zip(names, params)}))  # by value, not shared memory
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_allreduce_equals_full_batch(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    names, ref = _grads(_batch(16 * world, 0))
    for n, r in zip(names, ref):
        for rank in range(world):
            torch.testing.assert_close(torch.from_numpy(res[rank][n]), r, rtol=1e-4, atol=1e-6, msg=lambda m: f"{n} rank {rank}: {m}")


def _stage1_inputs(M, R, seed):
    g = torch.Generator().manual_seed(seed)
    return dict(pts=torch.randn(M, 3, generator=g), normals=torch.randn(M, 3, generator=g),
                flows=torch.randn(M, generator=g), weights=torch.rand(M, generator=g),
                flow_fw=(torch.rand(3, R, 2, generator=g) - 0.5) * 20.0,
                pix=torch.rand(R, 2, generator=g) * torch.tensor([31.0, 23.0]),
                ref=torch.rand(3, 3, 24, 32, generator=g), gt=torch.rand(R, 3, generator=g),
                omega=torch.randn(3, generator=g), vel=torch.randn(3, generator=g))


def _stage1_grads(inp, group=None):
    """Scene-flow loss + flow-RGB with their global normalisers (motion.py), the
    gradients of the motion velocities, the flows and the per-sample inputs."""
    from copenerf.motion import flow_rgb_loss, scene_flow_loss
    leaves = {k: v.clone().requires_grad_(True) for k, v in inp.items() if k in ("omega", "vel", "flow_fw", "normals",
                                                                                 "flows")}
    l_sf = scene_flow_loss(inp["pts"], leaves["normals"], leaves["flows"], inp["weights"], leaves["omega"],
                           leaves["vel"], group=group)
    l_fr = flow_rgb_loss(leaves["flow_fw"], inp["pix"], inp["ref"], inp["gt"], group=group).sum() / 3.0
    loss = 0.1 * l_sf + 7.5 * l_fr
    names = sorted(leaves)
    return names, torch.autograd.grad(loss, [leaves[k] for k in names])


def _stage1_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "cope-nerf_amd"), root, os.path.join(root, "tests")]
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from copenerf.train_step import flat_allreduce_mean
    S, R = 8, 16 * world
    full = _stage1_inputs(R * S, R, 1)
    r0, r1 = rank * 16, (rank + 1) * 16
    part = dict(full)
    for k in ("pts", "normals", "flows", "weights"):
        part[k] = full[k][r0 * S:r1 * S]
    part["flow_fw"], part["pix"], part["gt"] = full["flow_fw"][:, r0:r1], full["pix"][r0:r1], full["gt"][r0:r1]
    names, gr = _stage1_grads(part, group=dist.group.WORLD)
    # the shared leaves (ω, v) go through the flat all-reduce; the per-ray ones stay local
    shared = [torch.nn.Parameter(torch.zeros_like(g)) for n, g in zip(names, gr) if n in ("omega", "vel")]
    for p, g in zip(shared, [g for n, g in zip(names, gr) if n in ("omega", "vel")]):
        p.grad = g.clone()
    flat_allreduce_mean(shared)
    out = {n: g.numpy().copy() for n, g in zip(names, gr)}
    out["omega"], out["vel"] = shared[0].grad.numpy().copy(), shared[1].grad.numpy().copy()
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_stage1_global_normalisers():
    """Σw (scene-flow loss, train.py:477) and Σvalid (flow-RGB, train.py:515) are
    all-reduced before the divide: after the gradient all-reduce every rank has the
    single-process gradient of the shared motion velocities, and the per-ray input
    gradients equal world x the single-process ones (the mean over ranks divides them
    back) -- on 2 gloo ranks."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_stage1_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    S, R = 8, 16 * world
    names, ref = _stage1_grads(_stage1_inputs(R * S, R, 1))
    ref = dict(zip(names, ref))
    for rank in range(world):
        r0, r1 = rank * 16, (rank + 1) * 16
        for k in ("omega", "vel"):
            torch.testing.assert_close(torch.from_numpy(res[rank][k]), ref[k], rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(torch.from_numpy(res[rank]["normals"]) / world,
                                   ref["normals"][r0 * S:r1 * S], rtol=1e-5, atol=1e-8)
        torch.testing.assert_close(torch.from_numpy(res[rank]["flow_fw"]) / world, ref["flow_fw"][:, r0:r1],
                                   rtol=1e-5, atol=1e-8)
