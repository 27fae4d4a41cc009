"""GPU engine of the one-forward span format (serving/qa.py): batched prefill, no decode.

The span-pointer engine (:class:`~smsgate_amd.serving.engine.ExtractionEngine`) keeps a
KV slot per message for ~17 decode steps, replays decode hipGraphs, compacts rows and
harvests finished rows step by step.  A qa-format model answers in the forward that
reads the message, so serving it is a pipeline of packed prefill batches:

    host   take waiting messages (up to ``max_slots`` sequences / ``qa_max_tokens``
           tokens), append the query tokens, build positions / KV slots / pointer-row
           ids, stage them in ONE pinned copy
    GPU    embedding + pointer rows (embed_rows_add_ids) -> the native 30-layer prefill
           (csrc/runtime.hip, the same fused MFMA GEMM / attention kernels the span
           engine prefills with) -> qa_decode_kernel (query-row scores, class, joint
           constrained span decode, copy-format answer) -> async D2H of the answers
    host   harvest the PREVIOUS batch (its event) while this one runs

With ``qa_split_prefill`` > 0 a batch of that many tokens or more runs as two halves on
two streams (disjoint KV slots and output rows), one half's attention overlapping the
other's GEMMs as in the span engine's prefill; off by default (the ~220 k-row batches
fill the GPU alone: profiles/r05_qa_split_ab.jsonl).  The KV cache only lives for the batch: slot ``i`` is the
batch's ``i``-th sequence.

Same interface as the span engine for :class:`~smsgate_amd.serving.remote.EngineServer`
and :class:`~smsgate_amd.serving.worker.EngineWorker`: ``submit_ids`` / ``submit_many``,
``step(raw)`` returning ``(key, answer)`` or ``(key, copy-format token array)``,
``busy``, ``run``, ``stats``.  Plus :meth:`submit_packed`: a whole wire request (uint16
lengths + int32 ids) queued as ONE unit and answered as one :class:`PackedAnswer`, so
the engine server's Python work per request is a handful of numpy calls, not a few
objects and slices per message.
"""
from __future__ import annotations

import time
from collections import deque
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..models.extractor import SPAN_PTR0, ExtractorWeights
from ..models.tokenizer import ExtractorTokenizer
from ..parse.schema import EXTRACTOR_PROMPT
from .engine import EngineConfig, EngineStats, ExtractionEngine, _PinnedRing, _round_up
from .fsm import DEFAULT_FIELDS
from .protocol import PackedAnswer
from .qa import null_rejection, qa_layout, qa_token_flags

__all__ = ["QAEngine", "PackedAnswer"]


@dataclass
class _Join:
    """A request larger than the engine's slots, queued as several units: their answers
    are joined into one :class:`PackedAnswer` (in request order) when the last one lands."""
    parts: List[Optional[PackedAnswer]]
    left: int


@dataclass
class _Unit:
    """Queued work: one message (``packed`` False: ``submit_ids``) or a whole request."""
    key: Any
    lens: np.ndarray  # int32 [n] prompt lengths (capped)
    flat: np.ndarray  # int32 [sum(lens)] prompt ids
    packed: bool
    ntok: int = 0  # rows it adds to a batch (prompts + query tokens)
    join: Optional[_Join] = None  # part ``part`` of a split request
    part: int = 0


@dataclass
class _Batch:
    n: int
    units: List[_Unit]
    event: Any
    start_event: Any
    bufs: Dict[str, torch.Tensor]


class QAEngine(ExtractionEngine):
    """Prefill-only extraction engine of a qa-format model (``cfg.qa_queries > 0``)."""

    def __init__(self, weights: ExtractorWeights, tokenizer: ExtractorTokenizer,
                 cfg: Optional[EngineConfig] = None, system_prompt: str = EXTRACTOR_PROMPT) -> None:
        self.cfg = ec = cfg or EngineConfig()
        self.w = weights
        self.mc = mc = weights.cfg
        self.tok = tokenizer
        self.device = dev = weights.embed.device
        if dev.type != "cuda":
            raise RuntimeError("QAEngine needs a GPU (the HIP kernels have no CPU path)")
        if mc.qa_queries <= 0:
            raise ValueError("QAEngine serves qa-format models (ExtractorConfig.qa_queries > 0)")
        if mc.head_dim != 64 or mc.hidden % 64 or mc.inter % 32:
            raise ValueError("QAEngine: head_dim 64, hidden % 64 == 0, inter % 32 == 0 (fused kernels)")
        if mc.span_positions < ec.max_body_tokens + 2:
            raise ValueError("qa model: fewer pointer positions than prompt positions")
        if weights.embed.dtype != torch.bfloat16 or not weights.embed.is_contiguous():
            raise ValueError("QAEngine: contiguous bf16 weights")
        ops.load_library()
        ops.set_prefill_split(ec.prefill_key_split)
        ops.set_prefill_impl(ec.prefill_attn)
        self.lay = lay = qa_layout(SPAN_PTR0, mc.span_positions, mc.qa_queries, DEFAULT_FIELDS)
        if mc.vocab < lay.vocab:
            raise ValueError(f"qa model vocab {mc.vocab} < layout {lay.vocab}")
        self.NQ = lay.n_queries
        self.qids = np.asarray(lay.query_ids(), dtype=np.int32)
        # the span engine's state the shared helpers read (_compute_prefix, _layers_fused)
        self.fused, self.span, self.spec, self.copy, self.sparse, self.argmax = True, False, False, False, False, False
        self.template_slots = 0
        w = self.w
        self.fw_qkv = [ops.fold_norm(w.qkv[i], w.ln1[i]) for i in range(mc.layers)]
        self.fw_o = [w.o[i].contiguous() for i in range(mc.layers)]
        self.fw_gu = [ops.interleave_gate_up(ops.fold_norm(w.gate_up[i], w.ln2[i])) for i in range(mc.layers)]
        self.fw_down = [w.down[i].contiguous() for i in range(mc.layers)]
        # the head's rows (start pointers .. class rows) with the final norm folded in
        self.w_qa = ops.fold_norm(w.embed[lay.ptr0:lay.cls0 + 4], w.ln_f)
        self.flags_t = torch.from_numpy(qa_token_flags(tokenizer, lay.vocab).view(np.int32)).to(dev)
        self.params = ops.qa_params(lay, tokenizer, min_conf=ec.qa_min_conf)
        self.max_out = lay.max_answer_tokens()
        self.prefix_ids = tokenizer.prefix_ids(system_prompt)
        self.P0 = len(self.prefix_ids)
        self.P0pad = _round_up(self.P0, 32)
        self.Lmax = _round_up(ec.max_body_tokens + 2 + self.NQ, 32)
        S, L, nkv, D = ec.max_slots, mc.layers, mc.kv_heads, mc.head_dim
        bf = torch.bfloat16
        self.k_cache = torch.zeros(L, S, nkv, self.Lmax, D, dtype=bf, device=dev)
        self.vt_cache = torch.zeros(L, *ops.vt_shape(S, nkv, D, self.Lmax), dtype=bf, device=dev)
        self.pk = torch.zeros(L, nkv, self.P0pad, D, dtype=bf, device=dev)
        self.pvt = torch.zeros(L, *ops.vt_shape(1, nkv, D, self.P0pad)[1:], dtype=bf, device=dev)
        self.cos_sin = ops.rope_table(self.P0 + self.Lmax + 1, D, mc.rope_theta, dev)
        self.scale = 1.0 / (D ** 0.5)
        i32 = dict(dtype=torch.int32, device=dev)
        self.out_buf = torch.zeros(S, self.max_out, **i32)
        self.out_len = torch.zeros(S, **i32)
        self._host_bufs = [{"len": torch.zeros(S, dtype=torch.int32).pin_memory(),
                            "buf": torch.zeros(S, self.max_out, dtype=torch.int32).pin_memory()} for _ in range(2)]
        self._flip = 0
        self.max_tokens = max(ec.qa_max_tokens, ec.max_body_tokens + 2 + self.NQ)
        self._stage = _PinnedRing(max(1 << 20, 4 * (4 * self.max_tokens + 3 * S + 8)), slots=6)
        self.waiting: deque = deque()
        self.active: Dict[int, Any] = {}
        self.stats = EngineStats()
        self.graphs: Dict[int, Any] = {}
        self._inflight: deque = deque()  # launched, not yet harvested (oldest first; at most 2)
        self._sides: List[torch.cuda.Stream] = []
        self._fwd_ss: Optional[torch.Tensor] = None
        self._idle_prev = None
        self._idle_pairs: deque = deque()
        self._dbg: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None  # debug_decode's outputs
        self._lp = ops.LayerPointers(self.fw_qkv, self.fw_o, self.fw_gu, self.fw_down, self.k_cache, self.vt_cache,
                                     self.pk, self.pvt)
        self._compute_prefix()

    # ---------------------------------------------------------------- batches
    def _forward_part(self, lens: np.ndarray, ids: np.ndarray, r0: int) -> int:
        """Prefill + head of the messages ``lens`` / ``ids`` (int32, back to back) into KV
        slots / output rows ``r0 ..``; returns the tokens computed."""
        mc, lay, dev = self.mc, self.lay, self.device
        n = len(lens)
        NQ = self.NQ
        tl = lens + NQ
        T = int(tl.sum())
        cu = np.zeros(n + 1, dtype=np.int32)
        np.cumsum(tl, out=cu[1:])
        starts = np.repeat(cu[:-1], tl)
        pos = np.arange(T, dtype=np.int32) - starts
        in_msg = pos < np.repeat(lens, tl)
        # one concatenation of the messages, the query ids written around them
        flat = np.empty(T, dtype=np.int32)
        flat[in_msg] = ids
        flat[~in_msg] = np.tile(self.qids, n)
        add = np.where(in_msg, lay.ptr0 + pos, -1).astype(np.int32)
        seq_slot = np.arange(r0, r0 + n, dtype=np.int32)
        slot = np.repeat(seq_slot, tl)
        qstart = np.zeros(n, dtype=np.int32)
        trim = self.cfg.qa_trim_last and mc.layers > 1
        # the last layer on the query rows only: their indices, per-sequence row offsets
        # and key offsets (the body's length)
        qidx = (cu[1:, None] - NQ + np.arange(NQ, dtype=np.int32)[None, :]).reshape(-1)
        cuq = (NQ * np.arange(n + 1)).astype(np.int32)
        extra = [qidx, cuq, lens.astype(np.int32)] if trim else []
        meta = self._stage.to_device(np.concatenate([flat, pos, slot, add, cu, qstart, seq_slot] + extra), dev)
        o = 0
        flat_d = meta[o:o + T]; o += T
        pos_d = meta[o:o + T]; o += T
        slot_d = meta[o:o + T]; o += T
        add_d = meta[o:o + T]; o += T
        cu_d = meta[o:o + n + 1]; o += n + 1
        qstart_d = meta[o:o + n]; o += n
        seq_slot_d = meta[o:o + n]; o += n
        x = ops.embed_rows_add_ids(flat_d, add_d, self.w.embed)
        ss = self._ss_buffer(T, dev)
        H, I, nh, nkv, D = mc.hidden, mc.inter, mc.heads, mc.kv_heads, mc.head_dim
        q = torch.empty(T, nh, D, dtype=x.dtype, device=dev)
        ops.prefill_forward(self._lp, x, H=H, I=I, nh=nh, nkv=nkv, D=D,
                            Lmax=self.Lmax, P0=self.P0, P0pad=self.P0pad, pos=pos_d, slot=slot_d,
                            cos_sin=self.cos_sin, p0=self.P0, cu_q=cu_d, q_start=qstart_d, seq_slot=seq_slot_d,
                            max_q=int(tl.max()), scale=self.scale, q=q,
                            a=torch.empty(T, nh * D, dtype=x.dtype, device=dev),
                            act=torch.empty(T, I, dtype=x.dtype, device=dev), ss=ss, eps=mc.eps,
                            layers=mc.layers - 1 if trim else None)
        dbg = self._dbg if self._dbg is not None else (None, None, None)
        if not trim:
            ops.qa_decode(x, self.w_qa, mc.eps, cu_d, flat_d, self.flags_t, self.params, self.out_buf[r0:],
                          self.out_len[r0:], dbg[0], dbg[1], out_conf=dbg[2])
            return T
        Tq = n * NQ
        qidx_d = meta[o:o + Tq]; o += Tq
        cuq_d = meta[o:o + n + 1]; o += n + 1
        lens_d = meta[o:o + n]
        # last layer: K / V of every row (the query rows attend to the body), everything
        # else -- attention, o-proj, MLP -- for the query rows only (the body rows' last
        # hidden states are never read).  Same kernels and reduction orders per row as
        # the full layer, so the answers are the untrimmed ones (tests/test_qa_gpu.py).
        i = mc.layers - 1
        ops.gemm_qkv_rope(x, self.fw_qkv[i], mc.eps, pos_d, slot_d, self.cos_sin, q, self.k_cache[i],
                          self.vt_cache[i], nh, nkv, self.P0, cfg=ops.qkv_cfg(T, nh, nkv), ss_in=ss)
        a = torch.empty(Tq, nh * D, dtype=x.dtype, device=dev)
        ops.attn_prefill(q.index_select(0, qidx_d), cuq_d, lens_d, seq_slot_d, NQ, self.k_cache[i],
                         self.vt_cache[i], self.pk[i], self.pvt[i], self.P0, a, self.scale)
        xq = x.index_select(0, qidx_d)
        ssq = self._ss_buffer(Tq, dev)
        ops.gemm(a, self.fw_o[i], epi="resid", resid=xq, cfg=ops.gemm_cfg(Tq, H, epi="resid", K=nh * D),
                 ss_out=ssq)
        act = ops.gemm(xq, self.fw_gu[i], epi="swiglu", norm_eps=mc.eps,
                       out=torch.empty(Tq, I, dtype=x.dtype, device=dev),
                       cfg=ops.gemm_cfg(Tq, 2 * I, epi="swiglu", K=H), ss_in=ssq)
        ops.gemm(act, self.fw_down[i], epi="resid", resid=xq, cfg=ops.gemm_cfg(Tq, H, epi="resid", K=I))
        ops.qa_decode(xq, self.w_qa, mc.eps, cu_d, flat_d, self.flags_t, self.params, self.out_buf[r0:],
                      self.out_len[r0:], dbg[0], dbg[1], compact=True, out_conf=dbg[2])
        return T

    def submit_many(self, items) -> None:
        """Queue ``(key, body)`` pairs (tokenised here), one unit per message."""
        if items:
            self.submit_ids(list(zip((k for k, _ in items),
                                     self.tok.message_ids([b for _, b in items], self.cfg.max_body_tokens))))

    def submit_ids(self, items) -> None:
        """Queue pre-tokenised prompts (``body <ans>`` ids), one unit per message."""
        cap = self.cfg.max_body_tokens + 2
        for k, ids in items:
            a = np.asarray(ids, dtype=np.int32)
            if len(a) > cap:  # keep the closing <ans>
                a = np.concatenate([a[: cap - 1], a[-1:]])
            self.waiting.append(_Unit(k, np.asarray([len(a)], dtype=np.int32), a, False, len(a) + self.NQ))

    def submit_packed(self, key: Any, lens: np.ndarray, ids: np.ndarray) -> None:
        """Queue a whole request (wire lengths / ids); answered by :meth:`step` as
        ``(key, PackedAnswer)``.  Prompts over ``max_body_tokens + 2`` keep their first
        ``max_body_tokens + 1`` ids and their closing ``<ans>``.  A request of more
        prompts than ``max_slots`` is queued as several units and answered as one.
        Raises ``ValueError`` (nothing queued) for an empty prompt or lengths that do not
        add up to the ids: the wire is not trusted (a zero-length prompt would leave the
        decode kernel without a body to point into)."""
        lens = np.asarray(lens, dtype=np.int32)
        ids = np.asarray(ids, dtype=np.int32)
        if len(lens) and (int(lens.min()) < 1 or int(lens.sum(dtype=np.int64)) != len(ids)):
            raise ValueError(f"malformed request: {len(lens)} prompts, min length {int(lens.min())}, "
                             f"{int(lens.sum(dtype=np.int64))} ids declared, {len(ids)} sent")
        cap = self.cfg.max_body_tokens + 2
        if len(lens) and int(lens.max()) > cap:
            ends = np.cumsum(lens)
            keep = np.ones(len(ids), dtype=bool)
            for i in np.nonzero(lens > cap)[0].tolist():
                a, b = int(ends[i] - lens[i]), int(ends[i])
                keep[a + cap - 1:b - 1] = False
            ids, lens = ids[keep], np.minimum(lens, cap)
        S = self.cfg.max_slots
        if len(lens) <= S:
            self.waiting.append(_Unit(key, lens, ids, True, int(lens.sum()) + self.NQ * len(lens)))
            return
        k = -(-len(lens) // S)
        join = _Join([None] * k, k)
        ends = np.concatenate([[0], np.cumsum(lens, dtype=np.int64)])
        for j in range(k):
            a, b = j * S, min(len(lens), (j + 1) * S)
            part = lens[a:b]
            self.waiting.append(_Unit(key, part, ids[int(ends[a]):int(ends[b])], True,
                                      int(part.sum()) + self.NQ * len(part), join, j))

    def _launch(self) -> Optional[_Batch]:
        ec = self.cfg
        units: List[_Unit] = []
        n = ntok = 0
        S = ec.max_slots
        while self.waiting:
            u = self.waiting[0]
            m, t = len(u.lens), u.ntok
            if units and (n + m > S or ntok + t > self.max_tokens):
                break
            if m > S:  # the token budget is soft (a request larger than it runs alone); slots are not
                raise ValueError(f"a request of {m} prompts exceeds the engine's {S} slots")
            self.waiting.popleft()
            units.append(u)
            n += m
            ntok += t
        if not units:
            return None
        t0 = time.perf_counter()
        start_ev = None
        if ec.measure_idle:
            start_ev = torch.cuda.Event(enable_timing=True)
            start_ev.record()
        lens = np.concatenate([u.lens for u in units]) if len(units) > 1 else units[0].lens
        ids = np.concatenate([u.flat for u in units]) if len(units) > 1 else units[0].flat
        split = ec.qa_split_prefill
        if split and ntok >= split and n >= 2:
            h = n // 2
            o = int(lens[:h].sum())
            main = torch.cuda.current_stream(self.device)
            s2 = self._side_stream()
            s2.wait_stream(main)
            T = self._forward_part(lens[:h], ids[:o], 0)
            with torch.cuda.stream(s2):
                T += self._forward_part(lens[h:], ids[o:], h)
            main.wait_stream(s2)
        else:
            T = self._forward_part(lens, ids, 0)
        hb = self._host_bufs[self._flip]
        self._flip ^= 1
        hb["len"][:n].copy_(self.out_len[:n], non_blocking=True)
        hb["buf"][:n].copy_(self.out_buf[:n], non_blocking=True)
        ev = torch.cuda.Event(enable_timing=ec.measure_idle, blocking=True)
        ev.record()
        st = self.stats
        st.prefill_tokens += T
        st.prefill_seqs += n
        st.prefill_batches += 1
        st.prefill_s += time.perf_counter() - t0
        return _Batch(n, units, ev, start_ev, hb)

    def _harvest_batch(self, b: _Batch, raw: bool) -> List[Tuple[Any, Any]]:
        t0 = time.perf_counter()
        if not b.event.query():
            self._wait(b.event, float("inf"))
        lens = b.bufs["len"][: b.n].numpy().copy()
        blk = b.bufs["buf"][: b.n].numpy().copy()  # the pinned buffer is reused two batches on
        res: List[Tuple[Any, Any]] = []
        names = [f.name for f in DEFAULT_FIELDS]
        single: List[Tuple[Any, int]] = []
        r = 0
        for u in b.units:
            m = len(u.lens)
            if u.packed:
                ln = lens[r:r + m]
                keep = np.arange(blk.shape[1])[None, :] < ln[:, None]
                ans = PackedAnswer(ln.astype(np.uint16), blk[r:r + m][keep])
                if u.join is None:
                    res.append((u.key, ans))
                else:
                    u.join.parts[u.part] = ans
                    u.join.left -= 1
                    if u.join.left == 0:
                        parts = u.join.parts
                        res.append((u.key, PackedAnswer(np.concatenate([p.lens for p in parts]),
                                                        np.concatenate([p.flat for p in parts]))))
            elif raw:
                res.append((u.key, blk[r, : lens[r]]))
            else:
                single.append((u.key, r))
            r += m
        if single:
            rows = self.tok.decode_fields([blk[i, : lens[i]].tolist() for _, i in single], len(names))
            res += [(k, null_rejection(dict(zip(names, vals)))) for (k, _), vals in zip(single, rows)]
        self.stats.completed += b.n
        self.stats.harvest_s += time.perf_counter() - t0
        return res

    # -------------------------------------------------------------- scheduler
    def busy(self) -> bool:
        return bool(self.waiting or self._inflight)

    def _wait(self, ev, budget_s: float) -> bool:
        """Wait up to ``budget_s`` for ``ev`` without spinning a core: hipEventSynchronize
        (even on a blocking-sync event) kept the rank process busy-waiting, 12.7 of its
        17.9 us of CPU per message (profiles/r05_samples_top_bench.txt)."""
        t0 = time.perf_counter()
        done = ev.query()
        while not done and time.perf_counter() - t0 < budget_s:
            time.sleep(self.cfg.qa_poll_s)
            done = ev.query()
        self.stats.harvest_wait_s += time.perf_counter() - t0
        return done

    def step(self, raw: bool = False) -> List[Tuple[Any, Any]]:
        """Harvest every batch the GPU has finished, keep two batches in flight (the GPU
        runs batch k while the host stages k + 1 and decodes k - 1), and when neither is
        possible wait up to ``qa_wait_s`` for the oldest batch (then the caller -- the
        engine server -- polls its connections again).  Returns ``(key, answer)`` /
        ``(key, tokens)`` / ``(key, PackedAnswer)`` of the harvested work."""
        t0 = time.perf_counter()
        out: List[Tuple[Any, Any]] = []
        while self._inflight and self._inflight[0].event.query():
            out += self._harvest_batch(self._inflight.popleft(), raw)
        while self.waiting and len(self._inflight) < 2:
            # a second batch only once enough has queued: launching every trickle at once
            # (HTTP ingest) made batches of a few hundred rows, at a fraction of the
            # GPU's large-batch rate (profiles/r05_qa_engine_budget_sweep.jsonl)
            if self._inflight and sum(u.ntok for u in self.waiting) < self.cfg.qa_min_tokens:
                break
            new = self._launch()
            if new is None:
                break
            if self.cfg.measure_idle:
                if self._idle_prev is not None:
                    self._idle_pairs.append((self._idle_prev, new.start_event))
                self._idle_prev = new.event
            self._inflight.append(new)
        if not out and self._inflight and (len(self._inflight) >= 2 or not self.waiting
                                           or sum(u.ntok for u in self.waiting) < self.cfg.qa_min_tokens):
            if self._wait(self._inflight[0].event, self.cfg.qa_wait_s):
                out = self._harvest_batch(self._inflight.popleft(), raw)
        while self._idle_pairs and self._idle_pairs[0][1].query():
            a, b = self._idle_pairs.popleft()
            self.stats.gpu_idle_s += max(0.0, a.elapsed_time(b)) / 1000.0
        self.stats.steps += 1
        self.stats.step_s += time.perf_counter() - t0
        return out

    def debug_decode(self, msgs) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Tests: one synchronous batch of prompt ids (``body <ans>`` each) with the
        head's debug outputs -- the decoded (class, start, end ...) [M, 1 + 2 nf] int32
        (after abstention), the raw scores [M, 4 + nf (2 n_pos + 1)] fp32 and each
        answer's confidence [M] (ops.qa_decode)."""
        if self.busy():
            raise RuntimeError("debug_decode on a busy engine")
        cap = self.cfg.max_body_tokens + 2
        arrs = [np.asarray(m, dtype=np.int32) for m in msgs]
        arrs = [a if len(a) <= cap else np.concatenate([a[:cap - 1], a[-1:]]) for a in arrs]
        if not 0 < len(arrs) <= self.cfg.max_slots:
            raise ValueError("debug_decode: 1 .. max_slots prompts")
        M, nf, npos = len(arrs), self.lay.n_copy, self.lay.n_pos
        dev = self.device
        self._dbg = (torch.zeros(M, 4 + nf * (2 * npos + 1), dtype=torch.float32, device=dev),
                     torch.zeros(M, 1 + 2 * nf, dtype=torch.int32, device=dev),
                     torch.zeros(M, dtype=torch.float32, device=dev))
        try:
            self._forward_part(np.asarray([len(a) for a in arrs], dtype=np.int32), np.concatenate(arrs), 0)
            torch.cuda.synchronize(dev)
            sc, sp, cf = (t.cpu().numpy() for t in self._dbg)
        finally:
            self._dbg = None
        return sp, sc, cf
