"""Supervised training of the extractor LM on synthetic SMS (fwd + bwd on MI355X).

The reference never trains a model: it sends every SMS to Gemini
(libs/gemini_parser.py:273-292).  The local backend replaces that call with
our own extractor LM, and random-init weights only exercise
its speed.  This module turns the LM into a working extractor.

* data: :mod:`~smsgate_amd.utils.synth` bank SMS with ground-truth answers — the
  training template families (20 layouts in three languages; the held-out
  families are never seen),
  normalised exactly like the parse pipeline does before calling a backend
  (:func:`~smsgate_amd.parse.text.normalize_body`); skipped kinds (OTP, …) never
  reach the LLM and are not trained on;
* sequence: ``<bos> EXTRACTOR_PROMPT <sms>`` (shared) ``body <ans>`` followed by the
  compact answer (9 field values, each ended by ``<sep>``): the exact token
  stream the serving engine decodes.  Every target is checked against the
  schema FSM (:mod:`~smsgate_amd.serving.fsm`), so the constrained decoder can
  reproduce it;
* loss: next-token cross-entropy on the answer positions only, over the decode
  vocabulary (the tokenizer ids, the same rows the serving lm_head uses);
* model: fp32 master weights, bf16 autocast, AdamW with warmup + cosine decay; the
  served weights are an exponential moving average of the iterates (``ema``);
  The differentiable forward is :func:`~smsgate_amd.models.extractor.reference_forward`
  (PyTorch SDPA); serving uses the HIP kernels on the saved bf16 weights;
* data parallel: under ``torch.distributed`` (one process per GPU, RCCL) every
  rank draws its own examples and gradients are averaged by
  :class:`~smsgate_amd.parallel.ddp.GradBuckets` (flat buckets, all-reduce
  overlapped with backward); the global batch is ``batch x world``;
* checkpoint / resume: ``ckpt_dir`` gets ``step-XXXXXXX.pt`` (fp32 weights,
  optimizer state, step, data RNG state) every ``ckpt_every`` steps, written by
  rank 0 and loaded with ``torch.load(weights_only=True)``; ``resume=True``
  restarts from the newest one.
"""
from __future__ import annotations

import dataclasses
import math
import os
import random
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from ..parse.schema import EXTRACTOR_PROMPT
from ..parse.text import normalize_body
from .extractor import CONFIGS, SPAN_PTR0, ExtractorWeights, qa_config, reference_forward, span_config
from .tokenizer import ExtractorTokenizer, load_tokenizer

__all__ = ["TrainConfig", "FLAGSHIP_RECIPE", "recipe", "answer_tokens", "answer_span_tokens", "answer_fsm", "make_examples", "ExamplePool", "train_extractor", "field_accuracy",
           "latest_checkpoint", "to_serving", "qa_batch", "QASpec"]


@dataclass
class TrainConfig:
    model: str = "smollm-135m"
    steps: int = 1500
    batch: int = 64
    lr: float = 1e-3
    min_lr_frac: float = 0.05
    warmup: int = 100
    weight_decay: float = 0.01
    n_examples: int = 60000
    seed: int = 0
    max_body_tokens: int = 128
    log_every: int = 100
    ckpt_dir: Optional[str] = None
    ckpt_every: int = 0  # 0 = only at the end (when ckpt_dir is set)
    resume: bool = False
    bucket_mb: float = 64.0
    vocab_name: str = "train"  # synthetic vocabulary pool (utils.synth.vocab)
    # SMS layouts trained on: "train" = the training template families (utils.synth
    # TRAIN_FAMILIES, the two legacy formats included); None = the legacy mix only.
    # The held-out families (HELDOUT_FAMILIES) are never trained on.
    families: Optional[str] = "train"
    # exponential moving average of the weights (0 = off): the served weights are the
    # average over the last ~1/(1-ema) steps -- smoother than the last iterate, which
    # swings on SMS layouts it never saw from one checkpoint to the next
    ema: float = 0.998
    ema_start: int = 0  # first step the average includes (0 = warmup end)
    data_parallel: bool = True  # under torch.distributed: all-reduce gradients (False: train this rank alone)
    # data parallel with global_batch = batch x world: every rank holds the same example
    # list and draws the same global batch each step (the single-GPU run's stream), then
    # trains on its slice -- N ranks see exactly the examples one GPU would (0: each rank
    # draws its own batch from its own list)
    global_batch: int = 0
    # fused HIP RMSNorm / RoPE / SwiGLU forward+backward (models/train_ops.py) on the GPU;
    # False: reference_forward (plain PyTorch elementwise chains)
    fused: bool = True
    eval_every: int = 0  # call on_eval(step, serving weights) every N steps (0 = never)
    # "copy": every copied value written with the body's own tokens; "span": as two
    # pointers to its first and last body token (serving/fsm.py build_span_fsm)
    answer_format: str = "copy"
    # share of training examples drawn from the non-transaction families (utils/synth.py
    # NEG_TRAIN_FAMILIES: answer txn_type unknown / otp, every other field null)
    negatives: float = 0.12


# The ONE training recipe of the served extractor: bench.py's in-run
# training, ``python -m smsgate_amd train-extractor``'s defaults and the compose ``train``
# service all resolve to it (tests/test_deploy.py pins that), so the deployed model is
# the benchmarked one.  Fresh examples every step (n_examples = steps x global batch: a
# reused 60 k pool scored 87.4 vs 89.6 % held-out exact, profiles/r03_quality_probe.jsonl),
# 4 000 steps (6 000 did not help held-out formats, 96.5 vs 98.6 %,
# profiles/r05_qa_probe4_steps.jsonl), the one-forward qa answers, 12 % non-transactions,
# peak lr 5e-4 (round 6, widened value grammar: held-out formats 98.4 vs 94.4 % and
# training layouts 99.1 vs 96.8 % at 1e-3, mean of three samples each,
# profiles/r06d_qa_seeds.jsonl).  ``batch`` is the GLOBAL batch: data-parallel runs split
# it over the ranks (``global_batch``), so N GPUs train on the one-GPU run's batches.
FLAGSHIP_RECIPE = TrainConfig(model="smollm-135m", steps=4000, batch=128, lr=5e-4, n_examples=4000 * 128,
                              families="train", answer_format="qa", negatives=0.12, seed=0)


def recipe(model: Optional[str] = None, steps: Optional[int] = None, batch: Optional[int] = None,
           world: int = 1, **overrides) -> TrainConfig:
    """:data:`FLAGSHIP_RECIPE` with ``model`` / ``steps`` / global ``batch`` overridden
    (``n_examples`` follows: steps x batch fresh examples) and, for ``world`` > 1
    data-parallel ranks, the per-rank batch with ``global_batch`` set."""
    r = FLAGSHIP_RECIPE
    steps = r.steps if steps is None else steps
    batch = r.batch if batch is None else batch
    cfg = dataclasses.replace(r, model=model or r.model, steps=steps, batch=batch,
                              n_examples=overrides.pop("n_examples", 0) or steps * batch, **overrides)
    if world > 1:
        if batch % world:
            raise ValueError(f"global batch {batch} does not split over {world} ranks")
        cfg = dataclasses.replace(cfg, batch=batch // world, global_batch=batch, data_parallel=True)
    return cfg


def answer_tokens(tok: ExtractorTokenizer, fsm, answer: Dict[str, Optional[str]],
                  body: Optional[str] = None, body_enc=None) -> Optional[List[int]]:
    """Compact answer token ids, or None if the schema FSM cannot emit them (over a
    field's token cap, or a token outside the field's class).  With the (normalised)
    ``body`` each copied value is written with the body's own tokens
    (:meth:`ExtractorTokenizer.value_span_ids`); enum values use the FSM's trie."""
    ids: List[int] = []
    if body is not None and body_enc is None:
        body_enc = tok.encode_offsets([body])[0]
    for f in fsm.fields:
        v = answer.get(f.name) or ""
        if not v:
            vt: List[int] = []
        elif f.kind == "enum" or body is None:
            vt = tok.encode(v)
        else:
            vt = tok.value_span_ids(v, body, body_enc[0], body_enc[1])
        ids += vt + [tok.sep]
    state = fsm.start_state
    for t in ids:
        state = fsm.step_host(state, t)
        if state < 0:
            return None
    return ids if state == fsm.done_state else None


def answer_span_tokens(tok: ExtractorTokenizer, fsm, answer: Dict[str, Optional[str]], body: str, body_enc,
                       msg_len: int) -> Optional[List[int]]:
    """Span-format answer ids (enum tokens + <sep>; per copied field two pointers
    ``ptr0 + first``, ``ptr0 + last`` or <sep> when empty), or None when a value is no
    word-aligned body span inside the (truncated) message, or the FSM / copy rules
    reject it.  ``msg_len``: the message's ids incl. the closing <ans>."""
    ids: List[int] = []
    msg = list(body_enc[0][: msg_len - 1]) + [tok.ans]
    for f in fsm.fields:
        v = answer.get(f.name) or ""
        if f.kind == "enum":
            ids += (tok.encode(v) if v else []) + [tok.sep]
        elif not v:
            ids.append(tok.sep)
        else:
            sp = tok.value_span(v, body, body_enc[0], body_enc[1])
            if sp is None or sp[1] >= msg_len - 1:
                return None
            ids += [fsm.ptr0 + sp[0], fsm.ptr0 + sp[1]]
    state, prev = fsm.start_state, msg[-1]
    for t in ids:
        if not fsm.copy_mask_host(state, prev, msg)[t]:
            return None
        state, prev = fsm.step_host(state, t), t
    return ids if state == fsm.done_state else None


class QASpec:
    """The one-forward span format's training view (serving/qa.py): the id layout and
    the token flags its decoder checks gold spans against."""
    span = False
    qa = True

    def __init__(self, lay, flags) -> None:
        self.lay, self.flags = lay, flags

    @property
    def ptr0(self) -> int:
        return self.lay.ptr0

    @property
    def vocab(self) -> int:
        return self.lay.vocab

    @property
    def n_pos(self) -> int:
        return self.lay.n_pos


def answer_fsm(tok: ExtractorTokenizer, fmt: str = "copy", max_body: int = 128):
    """The schema FSM the training targets are written for (vocabulary trimmed to the
    tokenizer's ids, plus the pointer ids in span format)."""
    from ..serving.fsm import build_fsm, build_span_fsm, span_positions

    v_tok = (tok.vocab_size + 63) // 64 * 64
    if fmt in ("qa", "qa17"):
        from ..serving.qa import qa_layout, qa_token_flags

        # the engines (QAEngine, TorchQAExtractor) lay the pointer / query / class rows out
        # from SPAN_PTR0: a tokenizer of another size would train other rows than they serve
        assert v_tok == SPAN_PTR0, "the qa format's pointer ids follow the 8 192-id tokenizer"
        lay = qa_layout(v_tok, span_positions(max_body), 9 if fmt == "qa" else 17)
        return QASpec(lay, qa_token_flags(tok, lay.vocab))
    if fmt == "span":
        assert v_tok == SPAN_PTR0, "the span format's pointer ids follow the 8 192-id tokenizer"
        return build_span_fsm(tok, v_tok, span_positions(max_body))
    if fmt != "copy":
        raise ValueError(f"answer format {fmt!r}: copy | span | qa | qa17")
    return build_fsm(tok, v_tok)


def make_examples(tok: ExtractorTokenizer, fsm, n: int, seed: int,
                  max_body: int = 128, vocab_name: str = "train",
                  families: Optional[str] = "train", negatives: float = 0.0) -> List[Tuple[List[int], object]]:
    """``(message ids, answer)`` pairs (prefix excluded: it is shared): answer ids in the
    copy / span formats, ``(class, spans)`` in the qa format (serving/qa.py qa_targets).
    ``negatives``: share of non-transaction examples (``families`` must be a split)."""
    from ..utils.synth import HELDOUT_FAMILIES, generate, family_names

    if families is not None:
        assert not set(family_names(families)) & set(HELDOUT_FAMILIES), "held-out families are never trained on"
    out: List[Tuple[List[int], List[int]]] = []
    items = [s for s in generate(n, seed=seed, vocab_name=vocab_name, families=families, training=True,
                                 negatives=negatives if families is not None else 0.0)
             if s.answer is not None]
    bodies = [normalize_body(s.body) for s in items]
    msgs = tok.message_ids(bodies, max_body)
    encs = tok.encode_offsets(bodies)
    qa = getattr(fsm, "qa", False)
    if qa:
        from ..serving.qa import qa_targets
    for m, s, b, e in zip(msgs, items, bodies, encs):
        if qa:
            a = qa_targets(tok, fsm.lay, fsm.flags, s.answer, b, e, len(m))
        elif fsm.span:
            a = answer_span_tokens(tok, fsm, s.answer, b, e, len(m))
        else:
            a = answer_tokens(tok, fsm, s.answer, b, e)
        if a is not None:
            out.append((m, a))
    return out


_POOL_STATE: Dict[str, object] = {}


def _pool_init(tok_path: str, fmt: str = "copy", max_body: int = 128) -> None:
    tok = ExtractorTokenizer(Path(tok_path))
    _POOL_STATE["tok"] = tok
    _POOL_STATE["fsm"] = answer_fsm(tok, fmt, max_body)


def _pool_chunk(args) -> List[Tuple[List[int], object]]:
    n, seed, max_body, vocab_name, families, negatives = args
    return make_examples(_POOL_STATE["tok"], _POOL_STATE["fsm"], n, seed, max_body, vocab_name, families, negatives)


class ExamplePool:
    """Training examples built by CPU worker processes while the caller does other
    work (the bench starts it before the GPU is touched, then trains on the result).

    ``n`` examples in chunks of ``chunk``; chunk ``k`` is generated with seed
    ``seed * 7919 + k``, so the data depends only on (n, seed, chunk), never on the
    worker count.  The worker processes are spawned (not forked) and exit when the
    examples are collected."""

    def __init__(self, n: int, seed: int = 0, max_body: int = 128, vocab_name: str = "train",
                 families: Optional[str] = "train", workers: int = 8, chunk: int = 4096,
                 tok_path: Optional[str] = None, answer_format: str = "copy", negatives: float = 0.0) -> None:
        import multiprocessing as mp

        from .tokenizer import ASSET

        jobs = [(min(chunk, n - k * chunk), seed * 7919 + k, max_body, vocab_name, families, negatives)
                for k in range((n + chunk - 1) // chunk)]
        self.n = n
        self._pool = mp.get_context("spawn").Pool(max(1, min(workers, len(jobs))), initializer=_pool_init,
                                                  initargs=(str(tok_path or ASSET), answer_format, max_body))
        self._res = self._pool.map_async(_pool_chunk, jobs)

    def get(self, timeout: float = 1800.0) -> List[Tuple[List[int], List[int]]]:
        try:
            chunks = self._res.get(timeout)
        finally:
            self._pool.close()
            self._pool.join()
        return [e for c in chunks for e in c]


def _batch(prefix: List[int], exs: Sequence[Tuple[List[int], List[int]]], pad: int,
           device, ptr0: int = -1) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
    """ids, labels and (span format, ``ptr0 >= 0``) the pointer row added to each
    message position's input (-1 elsewhere)."""
    seqs = [prefix + m + a for m, a in exs]
    T = max(len(s) for s in seqs)
    ids = torch.full((len(seqs), T), pad, dtype=torch.long)
    labels = torch.full((len(seqs), T), -100, dtype=torch.long)
    add = torch.full((len(seqs), T), -1, dtype=torch.long) if ptr0 >= 0 else None
    P = len(prefix)
    for i, ((m, a), s) in enumerate(zip(exs, seqs)):
        ids[i, : len(s)] = torch.tensor(s)
        start = P + len(m)  # position of the first answer token
        labels[i, start - 1: start - 1 + len(a)] = torch.tensor(a)  # predicted from the previous position
        if add is not None:
            add[i, P:start] = torch.arange(ptr0, ptr0 + len(m))
    return ids.to(device), labels.to(device), (add.to(device) if add is not None else None)


def qa_batch(prefix: List[int], exs, pad: int, device, lay):
    """qa-format batch: ids ``prefix + message + queries``, the pointer row added to each
    message position (-1 elsewhere), the query rows' positions and the targets
    (class, starts, ends, pointable positions) of serving/qa.py qa_loss.  Built with
    numpy (one pass, no per-element tensor writes: the training step's host time)."""
    import numpy as np

    q = np.asarray(lay.query_ids(), dtype=np.int64)
    NQ, NF = len(q), lay.n_copy
    P = len(prefix)
    B = len(exs)
    lens = np.fromiter((len(m) for m, _ in exs), dtype=np.int64, count=B)
    T = P + int(lens.max()) + NQ
    ids = np.full((B, T), pad, dtype=np.int64)
    add = np.full((B, T), -1, dtype=np.int64)
    ids[:, :P] = prefix
    col = np.arange(T)[None, :]
    in_msg = (col >= P) & (col < P + lens[:, None])
    ids[in_msg] = np.concatenate([np.asarray(m, dtype=np.int64) for m, _ in exs])
    add[in_msg] = np.broadcast_to(lay.ptr0 + col - P, (B, T))[in_msg]
    qpos = P + lens[:, None] + np.arange(NQ)[None, :]
    ids[np.arange(B)[:, None], qpos] = q[None, :]
    t_cls = np.fromiter((c for _, (c, _) in exs), dtype=np.int64, count=B)
    sp = np.asarray([spans for _, (_, spans) in exs], dtype=np.int64).reshape(B, NF, 2)
    # one host->device copy for the whole batch (seven small ones cost ~0.5 ms of copy
    # engine time per step on the GPU: scripts/train_step_profile.py)
    parts = [ids, add, qpos, t_cls, sp[..., 0], sp[..., 1], lens - 1]
    flat = torch.from_numpy(np.concatenate([np.ascontiguousarray(a).reshape(-1) for a in parts])).to(device)
    out, o = [], 0
    for a in parts:
        out.append(flat[o:o + a.size].view(a.shape))
        o += a.size
    return out[0], out[1], out[2], tuple(out[3:])


def latest_checkpoint(ckpt_dir: Optional[str]) -> Optional[Path]:
    if not ckpt_dir or not os.path.isdir(ckpt_dir):
        return None
    cks = sorted(Path(ckpt_dir).glob("step-*.pt"))
    return cks[-1] if cks else None


def _save_checkpoint(ckpt_dir: str, step: int, w: ExtractorWeights, opt, rng: random.Random,
                     ema_params=None) -> Path:
    os.makedirs(ckpt_dir, exist_ok=True)
    path = Path(ckpt_dir) / f"step-{step:07d}.pt"
    tmp = path.with_suffix(".tmp")
    state = {"step": step, "weights": {k: v.detach().cpu() for k, v in w.state_dict().items()},
             "opt": opt.state_dict(), "rng": rng.getstate(), "model": w.cfg.name}
    if ema_params is not None:  # the running average is training state too (exact resume)
        state["ema"] = [e.detach().cpu() for e in ema_params]
    torch.save(state, tmp)
    os.replace(tmp, path)  # atomic: a crash never leaves a half-written "latest"
    return path


def to_serving(w: ExtractorWeights, cfg=None) -> ExtractorWeights:
    """bf16 inference copy of (fp32 master) weights.  Training runs on a vocab-trimmed
    copy of the architecture (only the tokenizer's ids exist); the serving copy has
    the full ``cfg.vocab`` embedding with the never-used rows zero (they are masked
    out of every decode step and no input id reaches them)."""
    cfg = cfg or w.cfg
    out = ExtractorWeights(cfg, device=w.embed.device, dtype=torch.bfloat16, seed=None)
    with torch.no_grad():
        for (n, p), (_, q) in zip(out.named_parameters(), w.named_parameters()):
            if n == "embed" and p.shape[0] != q.shape[0]:
                p.zero_()
                p[: q.shape[0]].copy_(q.to(torch.bfloat16))
            else:
                p.copy_(q.to(torch.bfloat16))
    out.requires_grad_(False)
    return out


def train_extractor(cfg: TrainConfig, device="cuda", log: Callable[[str], None] = print,
                    tok: Optional[ExtractorTokenizer] = None,
                    on_eval: Optional[Callable[[int, ExtractorWeights], None]] = None,
                    data: Optional[List[Tuple[List[int], List[int]]]] = None) -> ExtractorWeights:
    """Train and return **bf16** serving weights.  ``data``: prebuilt examples
    (e.g. :class:`ExamplePool`), else built here from ``cfg``."""
    import torch.distributed as dist

    from ..parallel.ddp import GradBuckets

    ddp = dist.is_initialized() and cfg.data_parallel
    rank = dist.get_rank() if ddp else 0
    world = dist.get_world_size() if ddp else 1

    tok = tok or load_tokenizer()
    mcfg = CONFIGS[cfg.model]
    fsm = answer_fsm(tok, cfg.answer_format, cfg.max_body_tokens)
    qa = getattr(fsm, "qa", False)
    if fsm.span:
        mcfg = span_config(mcfg, fsm.n_pos)
    elif qa:
        mcfg = qa_config(mcfg, fsm.n_pos, fsm.lay.n_queries)
    v_dec = min(mcfg.vocab, fsm.vocab)
    t0 = time.perf_counter()
    if data is None:
        data = make_examples(tok, fsm, cfg.n_examples, cfg.seed, cfg.max_body_tokens, cfg.vocab_name, cfg.families,
                             cfg.negatives)
    log(f"train: {len(data)} examples ({time.perf_counter() - t0:.1f}s), model {cfg.model}")
    prefix = tok.prefix_ids(EXTRACTOR_PROMPT)
    torch.manual_seed(cfg.seed)
    # train the architecture with its embedding trimmed to the ids the tokenizer can
    # produce (8192 of SmolLM's 49 152 rows): the other rows never get a gradient, so
    # carrying them through AdamW would only cost time (exact: see to_serving)
    tcfg = dataclasses.replace(mcfg, vocab=v_dec)
    w = ExtractorWeights(tcfg, device=device, dtype=torch.float32, seed=cfg.seed)
    decay = [p for n, p in w.named_parameters() if not n.startswith("ln")]
    no_decay = [p for n, p in w.named_parameters() if n.startswith("ln")]
    fused = str(device).startswith("cuda")  # one multi-tensor kernel per step instead of per-parameter ops
    opt = torch.optim.AdamW([{"params": decay, "weight_decay": cfg.weight_decay},
                             {"params": no_decay, "weight_decay": 0.0}], lr=cfg.lr, betas=(0.9, 0.95),
                            fused=fused)

    gb = GradBuckets(list(w.parameters()), bucket_mb=cfg.bucket_mb) if ddp else None
    params = list(w.parameters())
    ema_params = None
    ema_from = cfg.ema_start or cfg.warmup

    def lr_at(step: int) -> float:
        if step < cfg.warmup:
            return cfg.lr * (step + 1) / cfg.warmup
        p = (step - cfg.warmup) / max(1, cfg.steps - cfg.warmup)
        return cfg.lr * (cfg.min_lr_frac + (1 - cfg.min_lr_frac) * 0.5 * (1 + math.cos(math.pi * p)))

    shared = ddp and cfg.global_batch > 0
    if shared and cfg.global_batch != cfg.batch * world:
        raise ValueError(f"global_batch {cfg.global_batch} != batch {cfg.batch} x world {world}")
    # each rank draws its own examples, or (shared) every rank the single-GPU stream
    rng = random.Random(cfg.seed * 1000003 + (0 if shared else rank))
    start = 0
    ck = latest_checkpoint(cfg.ckpt_dir) if cfg.resume else None
    if ck is not None:
        state = torch.load(ck, map_location="cpu", weights_only=True)
        with torch.no_grad():
            for k, v in w.state_dict().items():
                v.copy_(state["weights"][k])
        opt.load_state_dict(state["opt"])
        start = int(state["step"])
        if "ema" in state:
            ema_params = [e.to(p.device) for e, p in zip(state["ema"], params)]
        if world == 1 or shared:
            rng.setstate(_as_rng_state(state["rng"]))
        else:  # rank 0's stream was saved; the others re-derive theirs deterministically
            rng = random.Random((cfg.seed * 1000003 + rank) ^ (start * 7919))
            if rank == 0:
                rng.setstate(_as_rng_state(state["rng"]))
        log(f"train: resumed from {ck} at step {start}")
    from . import train_ops

    if cfg.fused and train_ops.available(device):
        forward = train_ops.fused_forward
    else:
        def forward(w_, ids_, add_):
            return reference_forward(w_, ids_, compute_dtype=torch.float32, return_hidden=True, add_ids=add_)
    t0 = time.perf_counter()
    for step in range(start, cfg.steps):
        for g in opt.param_groups:
            g["lr"] = lr_at(step)
        if shared:
            exs_g = rng.sample(data, cfg.global_batch)
            exs = exs_g[rank * cfg.batch:(rank + 1) * cfg.batch]
        else:
            exs_g = exs = rng.sample(data, cfg.batch)
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=str(device).startswith("cuda")):
            if qa:
                from ..serving.qa import qa_logits, qa_loss

                ids, add, qpos, targets = qa_batch(prefix, exs, tok.pad, device, fsm.lay)
                h = forward(w, ids, add)
                # decisions of the (global) batch: class + a start per field + an end per
                # non-null field -- counted on the host, divided over the ranks
                n_dec = sum(1 + len(sp) + sum(1 for s_, _ in sp if s_ >= 0) for _, (_, sp) in exs_g)
                loss = qa_loss(qa_logits(h, w.embed, qpos, fsm.lay), targets, fsm.lay,
                               denom=n_dec / (world if shared else 1))
            else:
                ids, labels, add = _batch(prefix, exs, tok.pad, device, fsm.ptr0)
                h = forward(w, ids, add)
                sel = labels.view(-1) >= 0
                hs = h.reshape(-1, h.shape[-1])[sel]
                logits = hs @ w.embed[:v_dec].t()
                loss = F.cross_entropy(logits.float(), labels.view(-1)[sel])
        if gb is not None:
            gb.zero_grad()
            loss.backward()  # bucket all-reduces start as gradients land
            gb.finish()
        else:
            opt.zero_grad(set_to_none=True)
            loss.backward()
        torch.nn.utils.clip_grad_norm_(w.parameters(), 1.0)
        opt.step()
        if cfg.ema > 0 and step + 1 >= ema_from:
            with torch.no_grad():
                if ema_params is None:
                    ema_params = [p.detach().clone() for p in params]
                else:  # one multi-tensor lerp over all parameters
                    torch._foreach_lerp_(ema_params, [p.detach() for p in params], 1.0 - cfg.ema)
        if cfg.log_every and rank == 0 and (step % cfg.log_every == 0 or step == cfg.steps - 1):
            log(f"step {step:5d} loss {loss.item():.4f} lr {lr_at(step):.2e} ({time.perf_counter() - t0:.1f}s)"
                + (f" x{world} ranks" if world > 1 else ""))
        done = step + 1
        if on_eval is not None and cfg.eval_every and done % cfg.eval_every == 0 and done < cfg.steps:
            on_eval(done, to_serving(_with_ema(w, ema_params), mcfg))
        if cfg.ckpt_dir and rank == 0 and (done == cfg.steps or (cfg.ckpt_every and done % cfg.ckpt_every == 0)):
            _save_checkpoint(cfg.ckpt_dir, done, w, opt, rng, ema_params)
    return to_serving(_with_ema(w, ema_params), mcfg)


def _with_ema(w: ExtractorWeights, ema_params) -> ExtractorWeights:
    """``w`` itself, or a copy holding the averaged parameters."""
    if ema_params is None:
        return w
    out = ExtractorWeights(w.cfg, device=w.embed.device, dtype=torch.float32, seed=None)
    with torch.no_grad():
        for p, e in zip(out.parameters(), ema_params):
            p.copy_(e)
    return out


def _as_rng_state(st):
    """``random.Random.getstate()`` after a torch.save/load round trip (lists -> tuples)."""
    version, internal, gauss = st
    return (version, tuple(internal), gauss)


def field_accuracy(predicted: Sequence[Optional[Dict[str, Optional[str]]]],
                   expected: Sequence[Dict[str, Optional[str]]]) -> Dict[str, float]:
    """Exact-match rate per field and for whole answers."""
    fields = list(expected[0].keys()) if expected else []
    hits = {f: 0 for f in fields}
    whole = 0
    for p, e in zip(predicted, expected):
        ok = True
        for f in fields:
            same = p is not None and (p.get(f) or "") == (e.get(f) or "")
            hits[f] += same
            ok &= same
        whole += ok
    n = max(1, len(expected))
    res = {f: hits[f] / n for f in fields}
    res["all"] = whole / n
    return res
