"""Data-parallel training plumbing on CPU: bucketed all-reduce (gloo, 2 ranks) and
checkpoint / resume of the extractor trainer."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from smsgate_amd.models.extractor import CONFIGS, ExtractorWeights, reference_forward
from smsgate_amd.parallel.ddp import GradBuckets


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _loss(w, ids):
    logits = reference_forward(w, ids)
    return torch.nn.functional.cross_entropy(logits[:, :-1].reshape(-1, logits.shape[-1]), ids[:, 1:].reshape(-1))


def _worker(rank, world, port, bucket_mb, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    w = ExtractorWeights(CONFIGS["tiny"], dtype=torch.float32, seed=1)
    gb = GradBuckets(list(w.parameters()), bucket_mb=bucket_mb)
    g = torch.Generator().manual_seed(100 + rank)  # every rank has its own data
    ids = torch.randint(0, 8192, (2, 12), generator=g)
    # reference: per-rank local gradient, averaged with all_gather
    w.zero_grad(set_to_none=True)
    _loss(w, ids).backward()
    local = [p.grad.detach().clone() for p in w.parameters()]
    gathered = []
    for t in local:
        lst = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(lst, t)
        gathered.append(torch.stack(lst).mean(0))
    # bucketed path (hooks fire during backward)
    gb.zero_grad()
    _loss(w, ids).backward()
    gb.finish()
    ok = all(torch.allclose(p.grad, r, atol=1e-6, rtol=1e-5) for p, r in zip(w.parameters(), gathered))
    # two optimizer steps keep the replicas identical
    opt = torch.optim.AdamW(w.parameters(), lr=1e-3)
    for _ in range(2):
        gb.zero_grad()
        _loss(w, torch.randint(0, 8192, (2, 12), generator=g)).backward()
        gb.finish()
        opt.step()
    flat = torch.cat([p.detach().reshape(-1) for p in w.parameters()])
    lst = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(lst, flat)
    same = all(torch.equal(lst[0], x) for x in lst[1:])
    out[rank] = (ok, same, gb.num_buckets)
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb", [0.25, 64.0])
def test_bucketed_allreduce_matches_mean_and_keeps_replicas_identical(bucket_mb):
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), bucket_mb, out), nprocs=world, join=True)
    for r in range(world):
        ok, same, nb = out[r]
        assert ok, f"rank {r}: bucketed all-reduce != mean of local gradients"
        assert same, "replicas diverged"
        assert nb >= (2 if bucket_mb < 1 else 1)


def test_checkpoint_resume_is_exact(tmp_path):
    from smsgate_amd.models.train import TrainConfig, latest_checkpoint, train_extractor

    common = dict(model="tiny", batch=4, lr=1e-3, warmup=2, n_examples=300, log_every=0, max_body_tokens=48)
    full = train_extractor(TrainConfig(steps=4, **common), device="cpu", log=lambda *_: None)
    d = str(tmp_path / "ck")
    train_extractor(TrainConfig(steps=2, ckpt_dir=d, **common), device="cpu", log=lambda *_: None)
    assert latest_checkpoint(d).name == "step-0000002.pt"
    # a later run with the SAME schedule (steps=4) picks up at step 2
    resumed = train_extractor(TrainConfig(steps=4, ckpt_dir=d, resume=True, **common), device="cpu",
                              log=lambda *_: None)
    assert latest_checkpoint(d).name == "step-0000004.pt"
    for (n, a), (_, b) in zip(full.named_parameters(), resumed.named_parameters()):
        assert torch.equal(a, b), n


def test_torchrun_two_rank_training_cli(tmp_path):
    """``torchrun --nproc-per-node 2 -m smsgate_amd train-extractor`` on CPU (gloo):
    rank 0 writes the weights and the checkpoint; a --resume run continues from it."""
    import subprocess
    import sys

    out = tmp_path / "x.safetensors"
    ck = tmp_path / "ck"
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
            "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "-m", "smsgate_amd", "train-extractor",
            "--model", "tiny", "--batch", "4", "--examples", "300", "--out", str(out), "--ckpt-dir", str(ck)]
    env = dict(os.environ, LLM_DEVICE="cpu", OMP_NUM_THREADS="1")
    r = subprocess.run(base + ["--steps", "2"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert out.exists() and (ck / "step-0000002.pt").exists()
    r = subprocess.run(base + ["--steps", "3", "--resume"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "resumed from" in r.stdout + r.stderr and (ck / "step-0000003.pt").exists()


def _bench_worker(rank, world, port, cache, out):
    import sys

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = bench._args(["--model", "tiny", "--train-steps", "6", "--train-batch", "8", "--weights-cache", cache,
                        "--data-workers", "2"])
    pool = bench.start_training_data(args, rank)
    w, prov = bench.acquire_weights(args, "cpu", rank, world, pool)
    flat = torch.cat([p.detach().float().reshape(-1) for p in w.parameters()])
    lst = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(lst, flat)
    out[rank] = (all(torch.equal(lst[0], x) for x in lst[1:]), prov["weights"], w.cfg.qa_queries)
    dist.barrier()
    dist.destroy_process_group()


def test_bench_trains_data_parallel_on_every_rank(tmp_path):
    """with several ranks the bench's in-run training runs on ALL of
    them (the global batch split, gradients all-reduced) instead of local rank 0 while
    the others wait; the replicas end identical and rank 0 publishes the cache file."""
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_bench_worker, args=(world, _free_port(), str(tmp_path), out), nprocs=world, join=True)
    assert all(out[r][0] for r in range(world)), dict(out)
    assert all("data parallel over 2 ranks" in out[r][1] for r in range(world)), dict(out)
    assert out[0][2] == 9  # the default answer format (qa)
    assert len(list(tmp_path.glob("tiny-*.safetensors"))) == 1


def _single_worker(cache, out):
    import sys

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        os.environ.pop(k, None)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    args = bench._args(["--model", "tiny", "--train-steps", "6", "--train-batch", "8", "--weights-cache", cache,
                        "--data-workers", "2"])
    pool = bench.start_training_data(args, 0)
    w, _ = bench.acquire_weights(args, "cpu", 0, 1, pool)
    out[0] = torch.cat([p.detach().float().reshape(-1) for p in w.parameters()])


def _bench_flat_worker(rank, world, port, cache, out):
    import sys

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = bench._args(["--model", "tiny", "--train-steps", "6", "--train-batch", "8", "--weights-cache", cache,
                        "--data-workers", "2"])
    pool = bench.start_training_data(args, rank)
    w, _ = bench.acquire_weights(args, "cpu", rank, world, pool)
    if rank == 0:
        out[0] = torch.cat([p.detach().float().reshape(-1) for p in w.parameters()])
    dist.barrier()
    dist.destroy_process_group()


def test_bench_data_parallel_trains_the_one_gpu_model(tmp_path):
    """The N-rank job trains on the one-GPU job's global batches (every rank draws the
    same batch from the same example list and takes its slice).  Quality depends on the
    training sample (profiles/PERF.md, "Training determinism"), so the scaling runs must
    not train a different model at every N.  The weights match the single-process run up
    to the all-reduce's summation order."""
    single, multi = mp.Manager().dict(), mp.Manager().dict()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_single_worker, args=(str(tmp_path / "one"), single))
    p.start()
    p.join(600)
    assert p.exitcode == 0
    mp.spawn(_bench_flat_worker, args=(2, _free_port(), str(tmp_path / "two"), multi), nprocs=2, join=True)
    a, b = single[0], multi[0]
    rel = float((a - b).norm() / a.norm())
    print("relative weight difference, 2 ranks vs 1:", rel)
    assert rel < 1e-6, rel
