"""GPU extraction engine: continuous batching over a slot-resident KV cache.

One engine = one MI355X = one data-parallel replica (``smsgate_amd.parallel``).

Per engine:

* **weights** in serving layout (270 MB bf16 for the 135M extractor);
* **KV cache** ``K[L][slots][nkv][Lmax][D]`` and blocked ``V^T[L][slots][nkv][Lmax/8][D][8]``,
  zero-initialised, one fixed region per slot — at ~4.6 MB/slot (135M model,
  ``Lmax`` 200) thousands of concurrent sequences fit in 288 GB, so there is no
  paging/block-table indirection in the attention kernels;
* **shared prefix**: the system prompt (``<bos> EXTRACTOR_PROMPT``) is run
  once at start-up into ``pk``/``pvt``; every sequence attends to it without
  recomputing or copying it (and its K/V stay L2-resident across the batch);
* **per-row device state** (token, position, FSM state, done flag, output
  buffer) so the *whole* decode step — embedding → 30 layers → lm_head →
  FSM-masked sampling → state update — runs on the GPU without host
  round-trips, and ``steps_per_graph`` consecutive steps are captured into one
  hipGraph per batch-size bucket;
* **scheduler**: admit waiting requests into free rows (prefill packs many
  sequences into one varlen batch), replay decode graphs, harvest finished rows.

Hot ops are the HIP kernels of :mod:`smsgate_amd.ops`; the projections are
plain library GEMMs (hipBLASLt through ``torch.nn.functional.linear``).
"""
from __future__ import annotations

import heapq
import math
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Any, Deque, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops
from ..models.extractor import ExtractorConfig, ExtractorWeights
from ..models.tokenizer import ExtractorTokenizer
from ..parse.schema import EXTRACTOR_PROMPT
from .fsm import DEFAULT_FIELDS, FieldSpec, SchemaFSM, build_fsm, build_span_fsm
from .qa import null_rejection

__all__ = ["EngineConfig", "ExtractionEngine", "EngineStats"]


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# the served abstention threshold (EngineConfig.qa_min_conf, TorchQAExtractor)
QA_MIN_CONF = 0.0


@dataclass
class EngineConfig:
    max_slots: int = 1024
    max_body_tokens: int = 128
    temperature: float = 0.0
    seed: int = 0
    steps_per_graph: int = 4
    use_graphs: bool = True
    prefill_max_tokens: int = 32768
    admit_min_fraction: float = 0.25  # admit when this fraction of rows is free (or nothing runs)
    # admission batching at low load: while rows are decoding, hold arrivals until
    # `admit_min_batch` are waiting or the oldest has waited `admit_max_wait_s`
    # (one prefill of many short prompts costs about what a prefill of a few does); 0 = off.
    # Poisson A/B (profiles/r01c_admission_batching_ab.jsonl): p50 121 / 132 / 218 ms ->
    # 90 / 96 / 139 ms at 1 k / 2 k / 6 k msgs/s with 32 / 10 ms
    admit_min_batch: int = 32
    admit_max_wait_s: float = 0.01
    fused_gemm: bool = True  # csrc/gemm_kernels.hip (norm prologue, residual/SwiGLU epilogues) vs hipBLASLt
    compact: bool = True  # row compaction so the decode bucket tracks the active count
    decode_attn: str = "grouped"  # ops.attn_decode impl: grouped | cascade | mfma | mfma_v1 | valu | splitN
    # decode (sub-)batches of at most this many rows use `decode_attn_small` (key-split:
    # many short waves instead of few long ones — the low-load latency path); 0 = off.
    # kbench (profiles/r01c_kbench_small_buckets.json): split2 vs grouped 6.7 / 10.0 / 16.2
    # vs 15.8 / 18.3 / 20.5 us at 256 / 512 / 1024 rows, a tie at 2048, slower at 4096
    decode_attn_small_rows: int = 1024
    decode_attn_small: str = "split2"
    lm_head_fused: bool = False  # logits via the fused-norm GEMM instead of hipBLASLt (logits modes only)
    # greedy decoding: lm_head GEMM with the FSM-masked arg-max in its epilogue (EPI 4 of
    # csrc/gemm_kernels.hip) -- no [B, V] logits in HBM, no separate sampling kernel,
    # no vendor GEMM.  Needs temperature 0; sampling (temperature > 0) keeps the logits path.
    lm_head_argmax: bool = True
    buckets: Tuple[int, ...] = (64, 128, 256, 512, 1024, 2048, 4096, 8192)
    # nano-batch overlap (measured +10% msgs/s at 8192 slots, profiles/r01b_split_ab.txt):
    split_decode: int = 4096  # >0: decode buckets >= this run as two half-batches on two streams
    split_offset: bool = True  # start the second half one kernel behind the first
    split_graphs: int = 2  # 1 = both halves in one fork/join graph; 2 = one graph per part, one stream each
    split_parts: int = 2  # parts of a split decode bucket (split_graphs=2)
    split_prefill: int = 8192  # >0: prefill batches of >= this many tokens run as two halves on two streams
    prefill_key_split: int = 1  # 2: two waves share each prefill attention tile's keys (ops.set_prefill_split)
    prefill_attn: str = "auto"  # ops.set_prefill_impl: auto (= st32) / st / multi / per_head / gqa
    # speculative decoding (csrc/spec_kernels.hip): each decode step verifies up to
    # `spec_k` drafts per row looked up in the row's own SMS body (the extractor copies
    # body tokens); greedy only.  0 = off.  A step packs B rows + at most
    # ceil(spec_draft_frac * B) drafts into one forward (fixed shape per bucket).
    # measured (profiles/r02_bus_spec_ab.jsonl, r02_latency_trained_spec*.json): 2.54 tokens
    # per row-step on the trained 135M extractor, p50 latency 64 -> 33 ms at 1 k msgs/s,
    # 164 -> 76 ms at 10 k; +3-4 % msgs/s on the headline bench
    spec_k: int = 4
    spec_draft_frac: float = 1.25  # A/B 1.0 / 1.25 / 1.5 / 2.0: 22.5 / 23.2 / 23.1 / 21.5 k msgs/s
    spec_max_rows: int = 1 << 30  # buckets above this decode one token per row
    # verify attention: one wave per row reads the row's keys once for all its drafts
    # (ops.attn_spec; needs (1 + spec_k) * heads / kv_heads <= 32), else the decode kernel
    spec_attn: bool = True
    # draft policy (ops.spec_plan): 0 = copy the body until <sep>; 1 = + schema-forced
    # tokens, implicit value ends, copy across <sep> and from field starts.  1 emits
    # more tokens per row-step with an unlimited budget (scripts/spec_sim.py: 14.9 -> 11.8
    # steps/message) but its extra drafts are accepted less often, and under the
    # budget they displace better ones: 2.28 vs 2.40 tokens/row-step, 25.2 vs 26.0 k
    # msgs/s (profiles/r02_spec_policy_ab.jsonl)
    spec_policy: int = 0
    # RMSNorm row scales from the producer: the o-proj / down-proj GEMMs (residual
    # epilogue) also write per-tile sums of squares of the rows they store, and the
    # next norm GEMM (gate/up, QKV, lm_head arg-max) sums those partials instead of
    # accumulating x² with v_dot2 beside its MFMAs in every N tile (ops.gemm ss_out/ss_in)
    producer_norm: bool = True
    # copy-constrained decoding (serving/fsm.py FieldSpec.copy): in a copy field every
    # value token must be a body token, and after the first one a token that follows
    # the previous one somewhere in the body; applied per row in the lm_head arg-max
    # epilogue (ops.copy_masks -> gemm_argmax / fsm_sample / spec_verify)
    copy_constrain: bool = True
    # message-start templates: bank SMS open with a few fixed phrases ("APPROVED PURCHASE
    # DB SALE:", "DEBIT ACCOUNT\n" ...).  Causal attention makes the keys / values of a
    # body's first k tokens a function of those tokens alone, so a start shared by many
    # messages is computed ONCE into a template KV slot and copied into each matching
    # message's slot; its prefill starts at own offset k (ops.attn_prefill q_start).
    # Templates are learned from the traffic: the first k-token starts (2 <= k <=
    # template_max_len) of admitted bodies are counted, and every template_every
    # admissions those seen >= template_min_count times become templates (at most
    # template_slots).  0 slots = off.
    template_slots: int = 0
    template_max_len: int = 12
    template_min_count: int = 16
    template_every: int = 4096
    measure_idle: bool = True  # EngineStats.gpu_idle_s from two timing events per step
    # the prefill forward (not graph-captured: its shape changes with every admission)
    # launched by ONE native call (ops.prefill_forward, csrc/runtime.hip) instead of 150
    # Python wrapper calls per half batch (fused GEMM path only)
    native_prefill: bool = True
    # greedy copy-constrained decoding: the lm_head arg-max over each row's candidates only
    # (its body tokens / enum tokens, ops.sparse_argmax) instead of the dense 8 192-wide
    # GEMM with the masked arg-max epilogue (fused GEMM path, lm_head_argmax)
    sparse_argmax: bool = True
    # qa-format models (serving/qa_engine.py): token budget of one packed prefill batch
    # (messages + their query tokens; max_slots caps the sequences)
    qa_max_tokens: int = 262144
    # qa engine: a batch of >= this many tokens runs as two halves on two streams; 0 =
    # one prefill (profiles/r05_qa_split_ab.jsonl: 64.5 k msgs/s either way at the
    # ~220 k-row batches, so one stream, whose kernel times are not inflated by sharing)
    qa_split_prefill: int = 0
    # qa engine: how long one step() waits for the oldest in-flight batch before it
    # returns (the engine server then polls its connections), and the sleep between
    # event queries while it waits (no busy-wait on the host)
    # qa engine: the last layer only for the query rows (K / V of every row): the body
    # rows' last hidden states are never read
    qa_trim_last: bool = True
    # qa engine: rows that must be waiting before a SECOND batch is launched behind the
    # one in flight (the first always launches at once)
    qa_min_tokens: int = 65536
    # qa engine: abstention threshold -- a transaction answer whose confidence (its least
    # probable decision, serving/qa.py qa_confidence) is under this becomes "unknown"
    # (null fields: the reference's unmatched DLQ path) instead of being published with
    # a doubtful value; 0 = never abstain.  Calibrated on a validation set of TRAINING
    # layouts (profiles/PERF.md, "Abstention")
    qa_min_conf: float = QA_MIN_CONF
    qa_wait_s: float = 0.002
    qa_poll_s: float = 0.0002


@dataclass
class EngineStats:
    prefill_tokens: int = 0
    prefill_seqs: int = 0
    prefill_batches: int = 0  # qa engine: packed prefill launches
    prefill_s: float = 0.0
    template_tokens: int = 0  # prompt tokens NOT computed: copied from a message-start template
    templates: int = 0
    decode_steps: int = 0
    decode_row_steps: int = 0
    decode_s: float = 0.0
    harvest_s: float = 0.0
    harvest_wait_s: float = 0.0  # part of harvest_s blocked on the GPU (the snapshot's event)
    # GPU time with nothing queued between two steps (the host had not launched the next
    # step's work when the previous step's chunk finished): GPU-event timestamps, so it
    # measures starvation without a profiler (EngineConfig.measure_idle)
    gpu_idle_s: float = 0.0
    admit_s: float = 0.0
    compact_s: float = 0.0
    steps: int = 0
    step_s: float = 0.0  # wall time inside step() (the rest of a server loop is I/O)
    server_poll_s: float = 0.0  # EngineServer: receiving / unpacking / submitting requests
    server_send_s: float = 0.0  # EngineServer: packing / sending results
    compactions: int = 0
    rows_moved: int = 0
    completed: int = 0

    def as_dict(self) -> Dict[str, float]:
        return dict(self.__dict__)


@dataclass
class _Pending:
    key: Any
    ids: Any  # token ids: a list or an int32 array
    t: float = field(default_factory=time.perf_counter)  # arrival (admission batching)


@dataclass
class _Snapshot:
    B: int
    event: Any
    bufs: Dict[str, torch.Tensor]
    active: Dict[int, Any]  # row -> key at snapshot time (guards against re-admitted rows)


class _PinnedRing:
    """Persistent pinned host staging for host->device copies of index arrays.

    ``tensor.pin_memory()`` per call pins a fresh block every prefill / compaction
    (~23 ms a call when the rank process runs on few cores: profiles/r04_rank_pin_memory
    in PERF.md); here a ring of ``slots`` pre-pinned byte buffers is reused, each slot
    guarded by an event recorded after the copy that reads it, so a slot is rewritten
    only once its previous copy has finished (almost always already true)."""

    def __init__(self, nbytes: int, slots: int = 4) -> None:
        self.bufs = [torch.empty(nbytes, dtype=torch.uint8).pin_memory() for _ in range(slots)]
        self.events: List[Optional[torch.cuda.Event]] = [None] * slots
        self.k = 0

    def to_device(self, arr: np.ndarray, dev) -> torch.Tensor:
        arr = np.ascontiguousarray(arr)
        nb = arr.nbytes
        i = self.k
        self.k = (self.k + 1) % len(self.bufs)
        if nb > self.bufs[i].numel():  # larger than planned: grow this slot once
            if self.events[i] is not None:
                self.events[i].synchronize()
            self.bufs[i] = torch.empty(nb, dtype=torch.uint8).pin_memory()
        elif self.events[i] is not None:
            self.events[i].synchronize()
        host = self.bufs[i][:nb]
        host.numpy()[:] = arr.view(np.uint8).reshape(-1)
        out = host.view(_TORCH_DTYPE[arr.dtype.str]).view(arr.shape).to(dev, non_blocking=True)
        ev = torch.cuda.Event(blocking=True)
        ev.record()
        self.events[i] = ev
        return out


_TORCH_DTYPE = {"<i4": torch.int32, "<i8": torch.int64, "<f4": torch.float32}


class ExtractionEngine:
    def __init__(self, weights: ExtractorWeights, tokenizer: ExtractorTokenizer,
                 cfg: Optional[EngineConfig] = None, fields: Sequence[FieldSpec] = DEFAULT_FIELDS,
                 system_prompt: str = EXTRACTOR_PROMPT) -> None:
        self.cfg = cfg or EngineConfig()
        self.w = weights
        self.mc: ExtractorConfig = weights.cfg
        self.tok = tokenizer
        self.device = weights.embed.device
        if self.device.type != "cuda":
            raise RuntimeError("ExtractionEngine needs a GPU (the HIP kernels have no CPU path)")
        ops.load_library()
        mc, ec = self.mc, self.cfg
        ops.set_prefill_split(ec.prefill_key_split)  # process-wide launch settings
        ops.set_prefill_impl(ec.prefill_attn)
        if mc.head_dim != 64:
            raise ValueError("kernels are specialised for head_dim 64")
        # Constrained decoding can only ever emit tokenizer ids, so the lm_head is
        # evaluated on the first V_dec = roundup(tokenizer vocab, 32) rows of the
        # (tied) embedding: ids beyond it are masked in every FSM state, hence the
        # arg-max / Gumbel-max over allowed tokens is unchanged (exact, not an
        # approximation) and the projection is 6x smaller for the 49 152 vocab.
        self.V_dec = min(mc.vocab, _round_up(tokenizer.vocab_size, 64))
        # span-pointer models (models/extractor.py span_config): the pointer ids follow the
        # tokenizer's, and their rows are part of the lm_head
        span_fsm = (build_span_fsm(tokenizer, self.V_dec, mc.span_positions, fields)
                    if mc.span_positions > 0 else None)
        if span_fsm is not None:
            if mc.span_positions < ec.max_body_tokens + 2:
                raise ValueError("span model: fewer pointer positions than prompt positions")
            self.V_dec = span_fsm.vocab
        self.lm_head = self.w.embed[: self.V_dec]
        self.fused = ec.fused_gemm and self.V_dec % 64 == 0 and mc.hidden % 64 == 0 and mc.inter % 32 == 0
        if self.fused:
            # RMSNorm weights folded into the following projection; gate/up rows
            # interleaved in 16-row groups for the SwiGLU epilogue (ops.gemm).
            w = self.w
            self.fw_qkv = [ops.fold_norm(w.qkv[i], w.ln1[i]) for i in range(mc.layers)]
            self.fw_o = [w.o[i].contiguous() for i in range(mc.layers)]
            self.fw_gu = [ops.interleave_gate_up(ops.fold_norm(w.gate_up[i], w.ln2[i])) for i in range(mc.layers)]
            self.fw_down = [w.down[i].contiguous() for i in range(mc.layers)]
            self.fw_lm = ops.fold_norm(self.lm_head, w.ln_f)
        self.fsm: SchemaFSM = (span_fsm or build_fsm(tokenizer, self.V_dec, fields)).to_device(self.device)
        self.span = self.fsm.span
        self.argmax = ec.lm_head_argmax and ec.temperature <= 0 and self.V_dec % 128 == 0
        # out_buf holds the answer in copy format (a span answer is expanded by span_commit);
        # the KV cache holds the decode steps (2 pointers per field instead of its tokens)
        self.max_out = self.fsm.max_answer_tokens()
        self.prefix_ids = tokenizer.prefix_ids(system_prompt)
        self.P0 = len(self.prefix_ids)
        self.P0pad = _round_up(self.P0, 32)
        self.Lmax = _round_up(ec.max_body_tokens + 2 + self.fsm.max_steps(), 32)  # decode tiles are 32 keys
        if self.P0pad + self.Lmax > 512:
            raise ValueError("prefix + Lmax exceeds the decode kernel's context limit (512)")
        S, L, nkv, D = ec.max_slots, mc.layers, mc.kv_heads, mc.head_dim
        dev, bf = self.device, torch.bfloat16
        # span answers have nothing to draft: one pointer per step
        self.spec = ec.spec_k > 0 and ec.temperature <= 0 and not self.span
        self.copy = (ec.copy_constrain or self.span) and self.fsm.has_copy
        self.sparse = (ec.sparse_argmax and self.copy and self.argmax and self.fused
                       and ops.sparse_argmax_ok(self.fsm))
        if self.span and not self.sparse:
            raise ValueError("span-format models decode greedily through the fused sparse arg-max "
                             "(temperature 0, fused_gemm, lm_head_argmax, sparse_argmax)")
        if ec.spec_k > ops.SPEC_MAX_K:
            raise ValueError(f"spec_k <= {ops.SPEC_MAX_K}")
        self.template_slots = max(0, ec.template_slots)
        # speculative mode owns one extra scratch slot: unused pseudo-rows write their KV
        # there; template KV slots follow it (slot S + 1 + t)
        self.T0 = S + 1
        S_kv = S + 1 + self.template_slots if (self.spec or self.template_slots > 0) else S
        self.k_cache = torch.zeros(L, S_kv, nkv, self.Lmax, D, dtype=bf, device=dev)
        self.vt_cache = torch.zeros(L, *ops.vt_shape(S_kv, nkv, D, self.Lmax), dtype=bf, device=dev)
        self.pk = torch.zeros(L, nkv, self.P0pad, D, dtype=bf, device=dev)
        self.pvt = torch.zeros(L, *ops.vt_shape(1, nkv, D, self.P0pad)[1:], dtype=bf, device=dev)
        # cascade decode attention scratch: prefix output / log-sum-exp per query row
        self.attn_scratch = (torch.empty(S, mc.heads, D, dtype=torch.float32, device=dev),
                             torch.empty(S, mc.heads, dtype=torch.float32, device=dev))
        self.cos_sin = ops.rope_table(self.P0 + self.Lmax + 1, D, mc.rope_theta, dev)
        self.scale = 1.0 / math.sqrt(D)
        i32 = dict(dtype=torch.int32, device=dev)
        self.tok_buf = torch.zeros(S, **i32)
        self.pos = torch.zeros(S, **i32)
        self.state = torch.full((S,), self.fsm.done_state, **i32)
        self.done = torch.ones(S, **i32)
        self.out_len = torch.zeros(S, **i32)
        self.out_buf = torch.zeros(S, self.max_out, **i32)
        self.slot_id = torch.arange(S, **i32)  # row -> KV slot (rows are compacted, KV never moves)
        self.best = torch.zeros(S, dtype=torch.int64, device=dev)  # arg-max keys (lm_head_argmax)
        self.start_states = torch.full((S,), self.fsm.start_state, **i32)
        self.slot_host = np.arange(S, dtype=np.int32)
        self.free_rows: List[int] = list(range(S))
        heapq.heapify(self.free_rows)
        self.active: Dict[int, Any] = {}
        self.waiting: Deque[_Pending] = deque()
        self.stats = EngineStats()
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self._pool = None
        # double-buffered pinned host snapshots of the row state (see step())
        self._host_bufs = [
            {"done": torch.zeros(S, dtype=torch.int32).pin_memory(),
             "len": torch.zeros(S, dtype=torch.int32).pin_memory(),
             "buf": torch.zeros(S, self.max_out, dtype=torch.int32).pin_memory()}
            for _ in range(2)
        ]
        self._snap_flip = 0
        # pinned staging of the prefill / compaction index arrays (a prefill of T tokens
        # and n prompts stages 2T + 4n + 1 int32 + T int64)
        # 6 slots: a slot is reused only after the GPU has run the copy that reads it, so the
        # next admission may wait for the previous one's copies to come up in the stream; 32
        # slots removed that wait (admission host time 3.9 -> 1.5 s per phase) without a
        # throughput change outside the box-to-box spread (profiles/PERF.md, round 4)
        self._stage = _PinnedRing(max(1 << 20, 12 * ec.prefill_max_tokens + 16 * S + 64), slots=6)
        self._pending: Optional[_Snapshot] = None
        self._sides: List[torch.cuda.Stream] = []  # side streams of the split decode / prefill
        self._fwd_ss: Optional[torch.Tensor] = None  # row partials of the last forward's output (_layers_fused)
        self._idle_prev: Optional[Any] = None  # event after the last launched chunk (measure_idle)
        self._idle_pairs: Deque[Tuple[Any, Any]] = deque()  # (end of chunk k-1, start of step k) to price
        if self.spec or self.copy:
            # prompt ids per KV slot: the draft source and the copy constraint's body
            self.LB = ec.max_body_tokens + 2
            self.body_buf = torch.zeros(S_kv + 1, self.LB, **i32)
            self.body_len = torch.zeros(S_kv + 1, **i32)
        if self.copy:  # per-row copy masks of the one-token paths (prefill, plain decode)
            self.copy_rows = torch.zeros(S, self.V_dec // 32, **i32)
        if self.spec:
            self._init_spec()
        # message-start templates: tuple(first k ids) -> template slot; counts of starts
        self._tpl: Dict[Tuple[int, ...], int] = {}
        self._tpl_first: Dict[int, List[int]] = {}  # first token -> template lengths, longest first
        self._tpl_counts: Dict[Tuple[int, ...], int] = {}
        self._tpl_seen = 0
        # per-layer device addresses for the native prefill forward (the tensors above
        # never move: caches and weights are allocated once)
        self._lp = (ops.LayerPointers(self.fw_qkv, self.fw_o, self.fw_gu, self.fw_down, self.k_cache,
                                      self.vt_cache, self.pk, self.pvt)
                    if self.fused and ec.native_prefill else None)
        self._compute_prefix()
        if ec.use_graphs:
            self._capture_graphs()

    # ------------------------------------------------------------------ model
    def _layers(self, x: torch.Tensor, *, pos_tok: torch.Tensor, slot_tok: torch.Tensor, attn, k_cache,
                vt_cache, p0: int, hook=None) -> torch.Tensor:
        """Run all decoder layers on packed tokens; returns the final-normed hidden."""
        mc, w = self.mc, self.w
        T = x.shape[0]
        resid = x
        y: Optional[torch.Tensor] = None
        q = torch.empty(T, mc.heads, mc.head_dim, dtype=x.dtype, device=x.device)
        a = torch.zeros(T, mc.heads * mc.head_dim, dtype=x.dtype, device=x.device)  # (see _layers_fused)
        for i in range(mc.layers):
            h = ops.rmsnorm_residual(resid, w.ln1[i], mc.eps, x=y)
            qkv = F.linear(h, w.qkv[i])
            ops.rope_qkv_cache(qkv, pos_tok, slot_tok, self.cos_sin, q, k_cache(i), vt_cache(i), mc.heads,
                               mc.kv_heads, mc.head_dim, p0)
            if hook is not None:
                hook(i)
            attn(i, q, a)
            y = F.linear(a, w.o[i])
            h = ops.rmsnorm_residual(resid, w.ln2[i], mc.eps, x=y)
            act = ops.silu_mul(F.linear(h, w.gate_up[i]))
            y = F.linear(act, w.down[i])
        return ops.rmsnorm_residual(resid, w.ln_f, mc.eps, x=y)

    def _layers_fused(self, x: torch.Tensor, *, pos_tok: torch.Tensor, slot_tok: torch.Tensor, attn, k_cache,
                      vt_cache, p0: int, hook=None) -> torch.Tensor:
        """Same network with the fused MFMA GEMMs: ``x`` is the residual stream,
        updated in place; returns it UN-normed (the final norm is the lm_head
        GEMM's prologue, :meth:`_logits`)."""
        mc = self.mc
        T = x.shape[0]
        q = torch.empty(T, mc.heads, mc.head_dim, dtype=x.dtype, device=x.device)
        # ZEROED: the decode attention kernels skip finished rows, so their rows of `a`
        # would keep whatever the allocator's block held -- NaN bit patterns after training
        # ran in the same process -- and the next layer would write NaN keys / values into
        # their KV slots at their frozen positions.  A later message in that slot masks the
        # stale position inside its last key tile, but P = 0 times V = NaN is NaN: its
        # answer derails (the span bench's card-less answers, profiles/r04_span_template_runs.txt).
        a = torch.zeros(T, mc.heads * mc.head_dim, dtype=x.dtype, device=x.device)
        ss = self._ss_buffer(T, x.device)
        for i in range(mc.layers):
            # norm prologue + QKV projection + RoPE + KV-cache write: one kernel (layer 0's
            # input is the embedding: no producer, the GEMM accumulates x² itself)
            ops.gemm_qkv_rope(x, self.fw_qkv[i], mc.eps, pos_tok, slot_tok, self.cos_sin, q, k_cache(i),
                              vt_cache(i), mc.heads, mc.kv_heads, p0, ss_in=ss if i > 0 else None)
            if hook is not None:
                hook(i)
            attn(i, q, a)
            ops.gemm(a, self.fw_o[i], epi="resid", resid=x, ss_out=ss)
            act = ops.gemm(x, self.fw_gu[i], epi="swiglu", norm_eps=mc.eps, ss_in=ss)
            ops.gemm(act, self.fw_down[i], epi="resid", resid=x, ss_out=ss)
        self._fwd_ss = ss  # the final residual's row partials (the lm_head's norm)
        return x

    def _ss_buffer(self, T: int, dev) -> Optional[torch.Tensor]:
        """Zeroed fp32 [ops.SS_PARTS, T] row partials shared by one forward's residual-
        epilogue GEMMs, or None when both residual GEMMs would not tile N alike or
        would need more than SS_PARTS tiles (then every norm GEMM accumulates x² itself)."""
        if not self.cfg.producer_norm:
            return None
        mc = self.mc
        parts = {mc.hidden // ops.GEMM_TILES[ops.gemm_cfg(T, mc.hidden, epi="resid", K=k)][1]
                 for k in (mc.heads * mc.head_dim, mc.inter)}
        if len(parts) != 1 or parts.pop() > ops.SS_PARTS:
            return None
        return ops.ss_buffer(T, dev)

    def _embed(self, ids: torch.Tensor) -> torch.Tensor:
        """Input rows of int32 token ids (one gather kernel for bf16 weights)."""
        if self.w.embed.dtype == torch.bfloat16 and self.w.embed.is_contiguous():
            return ops.embed_rows(ids, self.w.embed)
        return F.embedding(ids.long(), self.w.embed)

    def _forward(self, x: torch.Tensor, **kw) -> torch.Tensor:
        return self._layers_fused(x, **kw) if self.fused else self._layers(x, **kw)

    def _argmax(self, h: torch.Tensor, row_state: torch.Tensor, best: torch.Tensor,
                ss: Optional[torch.Tensor] = None, row_masks: Optional[torch.Tensor] = None) -> torch.Tensor:
        """lm_head + FSM-masked arg-max keys (no logits materialised).  ``ss``: the
        forward's row partials of ``h`` (same rows), else the GEMM computes the norm;
        ``row_masks``: copy masks of the rows (:meth:`_copy_masks`)."""
        if self.fused:  # h is the un-normed residual stream: the final norm is the GEMM prologue
            return ops.gemm_argmax(h, self.fw_lm, row_state, self.fsm, best, norm_eps=self.mc.eps, ss_in=ss,
                                   row_masks=row_masks)
        return ops.gemm_argmax(h, self.lm_head, row_state, self.fsm, best, row_masks=row_masks)

    def _copy_masks(self, state: torch.Tensor, prev: torch.Tensor, slot: torch.Tensor,
                    out: torch.Tensor) -> Optional[torch.Tensor]:
        """Copy masks of rows in ``state`` whose last token is ``prev`` on KV ``slot``
        (None when copy-constrained decoding is off)."""
        if not self.copy:
            return None
        n = state.numel()
        return ops.copy_masks(self.fsm, state, prev, slot, self.body_buf, self.body_len, out[:n], n)

    def _logits(self, h: torch.Tensor) -> torch.Tensor:
        if self.fused:
            # measured (scripts/kbench.py, B=4096): hipBLASLt's 8192-wide lm_head
            # plus a separate RMSNorm beats the fused-norm GEMM at this width
            if self.cfg.lm_head_fused:
                return ops.gemm(h, self.fw_lm, norm_eps=self.mc.eps)
            h = ops.rmsnorm_residual(h, self.w.ln_f, self.mc.eps)
        return F.linear(h, self.lm_head)

    def _compute_prefix(self) -> None:
        ids = torch.tensor(self.prefix_ids, dtype=torch.int32, device=self.device)
        T = ids.numel()
        x = F.embedding(ids.long(), self.w.embed).contiguous()
        pos = torch.arange(T, dtype=torch.int32, device=self.device)
        slot = torch.zeros(T, dtype=torch.int32, device=self.device)
        cu = torch.tensor([0, T], dtype=torch.int32, device=self.device)
        qs = torch.zeros(1, dtype=torch.int32, device=self.device)
        s1 = torch.zeros(1, dtype=torch.int32, device=self.device)
        empty_k = torch.zeros(self.mc.kv_heads, 0, self.mc.head_dim, dtype=torch.bfloat16, device=self.device)
        empty_v = torch.zeros(self.mc.kv_heads, 0, self.mc.head_dim, 8, dtype=torch.bfloat16, device=self.device)

        def kc(i):
            return self.pk[i].unsqueeze(0)

        def vc(i):
            return self.pvt[i].unsqueeze(0)

        def attn(i, q, out):
            ops.attn_prefill(q, cu, qs, s1, T, kc(i), vc(i), empty_k, empty_v, 0, out, self.scale)

        self._forward(x, pos_tok=pos, slot_tok=slot, attn=attn, k_cache=kc, vt_cache=vc, p0=0)
        torch.cuda.synchronize(self.device)

    # ---------------------------------------------------------------- prefill
    def _prefill(self, rows: List[int], items: List[_Pending], sample: bool = True,
                 slots: Optional[np.ndarray] = None, templates: bool = True) -> torch.Tensor:
        """Prefill ``items`` into the KV slots of ``rows`` (or explicit ``slots``: a
        template fill, no row state) and sample their first answer token.  A body that
        opens with a message-start template gets the template's keys / values copied
        into its slot and is computed from own offset k on."""
        t0 = time.perf_counter()
        # vectorised host prep (runs while the previous decode chunk is on the GPU)
        n = len(items)
        full = np.fromiter((len(it.ids) for it in items), dtype=np.int32, count=n)
        dev = self.device
        seq_slots = self.slot_host[np.asarray(rows, dtype=np.int32)] if slots is None else slots.astype(np.int32)
        rows_np = np.asarray(rows if slots is None else np.zeros(n), dtype=np.int32)
        kk, tsl = self._match_templates(items) if (templates and self._tpl) else (None, None)
        skip = kk if kk is not None else np.zeros(n, dtype=np.int32)
        lens = full - skip
        T = int(lens.sum())
        flat = np.concatenate([it.ids[k:] for it, k in zip(items, skip.tolist())] if kk is not None
                              else [it.ids for it in items]).astype(np.int64, copy=False)
        cu = np.zeros(n + 1, dtype=np.int32)
        np.cumsum(lens, out=cu[1:])
        pos_np = np.arange(T, dtype=np.int32) - np.repeat(cu[:-1] - skip, lens)
        slot_np = np.repeat(seq_slots, lens)
        # one pinned staging copy for all small index arrays
        meta_d = self._stage.to_device(np.concatenate([pos_np, slot_np, cu, rows_np, full - 1, seq_slots, skip]), dev)
        o = 0
        pos_d = meta_d[o:o + T]; o += T
        slot_d = meta_d[o:o + T]; o += T
        cu_d = meta_d[o:o + n + 1]; o += n + 1
        rows_d = meta_d[o:o + n]; o += n
        last_pos_d = meta_d[o:o + n]; o += n
        seq_slot_d = meta_d[o:o + n]; o += n
        qstart = meta_d[o:o + n]
        if kk is not None:
            self._copy_templates(kk, tsl, seq_slots)
        if self.span and self.w.embed.dtype == torch.bfloat16 and self.w.embed.is_contiguous():
            # prompt position j also carries pointer j's row: one fused gather + add
            flat_d = self._stage.to_device(flat.astype(np.int32), dev)
            x = ops.embed_rows_add(flat_d, pos_d, self.w.embed, self.fsm.ptr0)
        else:
            flat_d = self._stage.to_device(flat, dev)
            x = F.embedding(flat_d, self.w.embed)
            if self.span:
                x = x + F.embedding(pos_d.long() + self.fsm.ptr0, self.w.embed)
            x = x.contiguous()
        max_q = int(lens.max())
        if self.spec or self.copy:  # the rows' prompts: draft source and copy set
            self.body_buf[slot_d.long(), pos_d.long()] = flat_d.to(torch.int32)
            self.body_len[seq_slot_d.long()] = last_pos_d + 1

        def kc(i):
            return self.k_cache[i]

        def vc(i):
            return self.vt_cache[i]

        def attn(i, q, out):
            ops.attn_prefill(q, cu_d, qstart, seq_slot_d, max_q, kc(i), vc(i), self.pk[i], self.pvt[i], self.P0, out,
                             self.scale)

        if self._lp is not None:
            mc = self.mc
            ss = self._ss_buffer(T, dev)
            ops.prefill_forward(self._lp, x, H=mc.hidden, I=mc.inter, nh=mc.heads, nkv=mc.kv_heads, D=mc.head_dim,
                                Lmax=self.Lmax, P0=self.P0, P0pad=self.P0pad, pos=pos_d, slot=slot_d,
                                cos_sin=self.cos_sin, p0=self.P0, cu_q=cu_d, q_start=qstart, seq_slot=seq_slot_d,
                                max_q=max_q, scale=self.scale,
                                q=torch.empty(T, mc.heads, mc.head_dim, dtype=x.dtype, device=dev),
                                a=torch.empty(T, mc.heads * mc.head_dim, dtype=x.dtype, device=dev),
                                act=torch.empty(T, mc.inter, dtype=x.dtype, device=dev), ss=ss, eps=mc.eps)
            self._fwd_ss = ss
            h = x
        else:
            h = self._forward(x, pos_tok=pos_d, slot_tok=slot_d, attn=attn, k_cache=kc, vt_cache=vc, p0=self.P0)
        if slots is not None:  # a template fill: its keys / values are all it leaves
            return None
        last = h.index_select(0, (cu_d[1:] - 1).long())
        if not sample or not self.argmax:
            logits = self._logits(last)
        if not sample:
            return logits
        # reset the admitted rows, then sample their first answer token
        rl = rows_d.long()
        self.done.index_fill_(0, rl, 0)
        self.out_len.index_fill_(0, rl, 0)
        self.state.index_fill_(0, rl, self.fsm.start_state)
        self.pos.index_copy_(0, rl, last_pos_d)
        cm = None
        if self.copy and not self.sparse and int(self.fsm.copy_kind[self.fsm.start_state]):
            # a first field that copies: every body token may start it (prev is unused)
            # (own buffer: the two halves of a split prefill run concurrently)
            cm = self._copy_masks(self.start_states[:n], self.start_states[:n], seq_slot_d,
                                  torch.empty(n, self.V_dec // 32, dtype=torch.int32, device=dev))
        if self.argmax:
            best = torch.empty(n, dtype=torch.int64, device=dev)
            if self.sparse:
                ops.sparse_argmax(last, self.fw_lm, self.start_states[:n], self.fsm, best, self.start_states[:n],
                                  seq_slot_d, self.body_buf, self.body_len, self.mc.eps)
            else:
                self._argmax(last, self.start_states[:n], best, row_masks=cm)
            if self.span:
                ops.span_commit(best, self.fsm, self.state, self.tok_buf, self.out_buf, self.out_len, self.done,
                                self.pos, seq_slot_d, self.body_buf, self.body_len, n, row_map=rows_d)
            else:
                ops.fsm_commit(best, self.fsm, self.state, self.tok_buf, self.out_buf, self.out_len, self.done,
                               self.pos, n, row_map=rows_d)
            logits = None
        else:
            ops.fsm_sample(logits, self.fsm, self.state, self.tok_buf, self.out_buf, self.out_len, self.done,
                           self.pos, self.slot_id, self.cfg.temperature, self.cfg.seed, row_map=rows_d, row_masks=cm)
        self.stats.prefill_tokens += T
        self.stats.prefill_seqs += len(items)
        self.stats.template_tokens += int(skip.sum())
        self.stats.templates = len(self._tpl)
        self.stats.prefill_s += time.perf_counter() - t0
        return logits

    # ----------------------------------------------------- message-start templates
    def _match_templates(self, items: List[_Pending]) -> Tuple[Optional[np.ndarray], Optional[np.ndarray]]:
        """Longest template opening each body: (k, template slot) per item, or (None,
        None) when no item matches.  A match leaves >= 1 token (the <ans>) to compute."""
        n = len(items)
        kk = np.zeros(n, dtype=np.int32)
        tsl = np.zeros(n, dtype=np.int32)
        hit = False
        first = self._tpl_first
        for i, it in enumerate(items):
            ids = it.ids
            for k in first.get(int(ids[0]), ()):  # this first token's template lengths, longest first
                if k < len(ids):
                    t = self._tpl.get(tuple(ids[:k]))
                    if t is not None:
                        kk[i], tsl[i] = k, t
                        hit = True
                        break
        return (kk, tsl) if hit else (None, None)

    def _copy_templates(self, kk: np.ndarray, tsl: np.ndarray, seq_slots: np.ndarray) -> None:
        """Copy each matching item's template keys / values (own offsets 0..k-1, every
        layer) and prompt ids into its slot.  Rows past an item's own k carry template
        padding that the item's prefill overwrites (it writes offsets >= k)."""
        sel = np.nonzero(kk)[0]
        kmax = int(kk[sel].max())
        dev = self.device
        items = self._stage.to_device(np.stack([tsl[sel], seq_slots[sel], kk[sel]]).astype(np.int32), dev)
        # exactly k rows per item, every layer, one launch (a torch gather / index_put of
        # the kmax-row block of all layers moved ~0.3 GB per admitted batch and cost more
        # than the prefill rows it saved: profiles/r03_ab_templates.jsonl)
        ops.kv_copy_prefix(self.k_cache, self.vt_cache, items)
        if self.spec or self.copy:
            src, dst = items[0].long(), items[1].long()
            self.body_buf[dst, :kmax] = self.body_buf[src, :kmax]

    def _learn_templates(self, items: Sequence[_Pending]) -> None:
        """Count the k-token starts of admitted bodies; every ``template_every``
        admissions promote the most frequent (count x k, >= template_min_count) to
        template slots and compute their keys / values (one small prefill)."""
        ec = self.cfg
        if self.template_slots <= 0 or len(self._tpl) >= self.template_slots:
            return
        cnt = self._tpl_counts
        kmax = ec.template_max_len
        for it in items:
            ids = it.ids
            for k in range(2, min(kmax, len(ids) - 1) + 1):
                key = tuple(ids[:k])
                cnt[key] = cnt.get(key, 0) + 1
        self._tpl_seen += len(items)
        if self._tpl_seen < ec.template_every:
            return
        self._tpl_seen = 0
        cands = sorted((c * len(key), key) for key, c in cnt.items()
                       if c >= ec.template_min_count and key not in self._tpl)
        new = []
        while cands and len(self._tpl) + len(new) < self.template_slots:
            new.append(cands.pop()[1])
        if new:
            slots = np.arange(len(self._tpl), len(self._tpl) + len(new), dtype=np.int32) + self.T0
            # a template's own keys depend only on its tokens: prefill them alone
            self._prefill([], [_Pending(None, list(key)) for key in new], sample=False, slots=slots,
                          templates=False)
            for key, sl in zip(new, slots.tolist()):  # (the fill wrote their ids to body_buf too)
                self._tpl[key] = sl
            first: Dict[int, set] = {}
            for key in self._tpl:
                first.setdefault(int(key[0]), set()).add(len(key))
            self._tpl_first = {t: sorted(ks, reverse=True) for t, ks in first.items()}
            self.stats.templates = len(self._tpl)
        self._tpl_counts = {}  # a fresh window: the next promotion sees recent traffic

    # ----------------------------------------------------------------- decode
    def _decode_step(self, B: int, sample: bool = True, r0: int = 0, hook=None) -> torch.Tensor:
        """One decode step of rows ``r0 .. r0+B`` (every per-row buffer is sliced,
        so two disjoint row ranges can run as independent sub-batches)."""
        if sample and self._use_spec(B):  # (debug_logits wants one plain token per row)
            return self._spec_step(B, r0, hook=hook, sample=sample)
        r1 = r0 + B
        tok = self.tok_buf[r0:r1]
        pos = self.pos[r0:r1]
        slot = self.slot_id[r0:r1]
        done = self.done[r0:r1]
        scratch = (self.attn_scratch[0][r0:r1], self.attn_scratch[1][r0:r1])
        x = self._embed(tok)
        impl = self.cfg.decode_attn_small if B <= self.cfg.decode_attn_small_rows else self.cfg.decode_attn

        def kc(i):
            return self.k_cache[i]

        def vc(i):
            return self.vt_cache[i]

        def attn(i, q, out):
            ops.attn_decode(q, pos, slot, kc(i), vc(i), self.pk[i], self.pvt[i], self.P0, out, self.scale,
                            done=done, impl=impl, scratch=scratch)

        h = self._forward(x, pos_tok=pos, slot_tok=slot, attn=attn, k_cache=kc, vt_cache=vc, p0=self.P0,
                          hook=hook)
        cm = (self._copy_masks(self.state[r0:r1], tok, slot, self.copy_rows[r0:r1])
              if sample and self.copy and not self.sparse else None)
        if sample and self.argmax:
            best = self.best[r0:r1]
            if self.sparse:
                ops.sparse_argmax(h, self.fw_lm, self.state[r0:r1], self.fsm, best, tok, slot, self.body_buf,
                                  self.body_len, self.mc.eps)
            else:
                self._argmax(h, self.state[r0:r1], best, ss=self._fwd_ss if self.fused else None, row_masks=cm)
            if self.span:
                ops.span_commit(best, self.fsm, self.state[r0:r1], tok, self.out_buf[r0:r1], self.out_len[r0:r1],
                                done, pos, slot, self.body_buf, self.body_len, B)
            else:
                ops.fsm_commit(best, self.fsm, self.state[r0:r1], tok, self.out_buf[r0:r1], self.out_len[r0:r1],
                               done, pos, B)
            return best
        logits = self._logits(h)
        if sample:
            ops.fsm_sample(logits, self.fsm, self.state[r0:r1], tok, self.out_buf[r0:r1], self.out_len[r0:r1],
                           done, pos, slot, self.cfg.temperature, self.cfg.seed, row_masks=cm)
        return logits

    # ----------------------------------------------------------- speculative
    def _init_spec(self) -> None:
        ec, dev = self.cfg, self.device
        S = ec.max_slots
        i32 = dict(dtype=torch.int32, device=dev)
        self.scratch_slot = S
        # tokens that end a copied value in the body: drafted as <sep>
        strings = self.tok.token_strings
        delim = [(("," in t) or ("&#" in t) or (";" in t)) and i not in (self.tok.sep,) for i, t in enumerate(strings)]
        delim += [False] * (self.V_dec - len(delim))
        self.spec_delim = torch.tensor(delim[: self.V_dec], dtype=torch.uint8, device=dev)
        self._spec_mult = 1 + math.ceil(ec.spec_draft_frac)
        self.draft_buf = torch.zeros(S * ops.SPEC_MAX_K, **i32)
        cap = S * self._spec_mult
        self.x_tok = torch.zeros(cap, **i32)
        self.x_pos = torch.zeros(cap, **i32)
        self.x_slot = torch.full((cap,), S, **i32)
        self.x_done = torch.ones(cap, **i32)
        self.x_state = torch.full((cap,), self.fsm.done_state, **i32)
        self.x_best = torch.zeros(cap, dtype=torch.int64, device=dev)
        if self.copy:  # one copy mask per pseudo-row
            self.copy_x = torch.zeros(cap, self.V_dec // 32, **i32)
        self.row_start = torch.zeros(S, **i32)
        self.row_nd = torch.zeros(S, **i32)
        self.spec_acc = torch.zeros(S, **i32)
        self.spec_meta = torch.zeros(S, **i32)  # [r0] = pseudo-rows used by the part starting at row r0
        self.spec_counts = torch.zeros(2, dtype=torch.int64, device=dev)  # [tokens emitted, live row-steps]

    def _tcap(self, B: int) -> int:
        """Pseudo-rows of a speculative step over ``B`` rows (drafts capped at the budget)."""
        d = min(_round_up(math.ceil(B * self.cfg.spec_draft_frac), 64), B * (self._spec_mult - 1))
        return B + d

    def _use_spec(self, B: int) -> bool:
        return self.spec and B <= self.cfg.spec_max_rows

    def _spec_step(self, B: int, r0: int = 0, hook=None, sample: bool = True) -> torch.Tensor:
        """One speculative decode step of rows ``r0 .. r0+B``: plan (drafts + packing),
        verify forward over the pseudo-rows, greedy FSM verification."""
        r1 = r0 + B
        T = self._tcap(B)
        off = r0 * self._spec_mult
        tok, pos, slot, done = self.tok_buf[r0:r1], self.pos[r0:r1], self.slot_id[r0:r1], self.done[r0:r1]
        xt, xp, xs, xd = (self.x_tok[off:off + T], self.x_pos[off:off + T], self.x_slot[off:off + T],
                          self.x_done[off:off + T])
        rs, nd, acc = self.row_start[r0:r1], self.row_nd[r0:r1], self.spec_acc[r0:r1]
        xst = self.x_state[off:off + T]
        ops.spec_plan(self.fsm, self.state[r0:r1], xst, self.cfg.spec_k, T, self.tok.sep, self.scratch_slot, tok,
                      pos, slot, done,
                      self.out_buf[r0:r1], self.out_len[r0:r1], self.body_buf, self.body_len, self.spec_delim,
                      self.draft_buf[r0 * ops.SPEC_MAX_K:], xt, xp, xs, xd, rs, nd, self.spec_meta[r0:r0 + 1],
                      policy=self.cfg.spec_policy)
        x = self._embed(xt)
        impl = self.cfg.decode_attn_small if T <= self.cfg.decode_attn_small_rows else self.cfg.decode_attn
        scratch = None
        if impl == "cascade":
            scratch = (torch.empty(T, self.mc.heads, self.mc.head_dim, dtype=torch.float32, device=self.device),
                       torch.empty(T, self.mc.heads, dtype=torch.float32, device=self.device))

        def kc(i):
            return self.k_cache[i]

        def vc(i):
            return self.vt_cache[i]

        max_q = 1 + self.cfg.spec_k
        if self.cfg.spec_attn and max_q * (self.mc.heads // self.mc.kv_heads) <= 32:
            def attn(i, q, out):
                ops.attn_spec(q, rs, nd, xp, xs, xd, kc(i), vc(i), self.pk[i], self.pvt[i], self.P0, out,
                              self.scale, max_q)
        else:
            def attn(i, q, out):
                ops.attn_decode(q, xp, xs, kc(i), vc(i), self.pk[i], self.pvt[i], self.P0, out, self.scale,
                                done=xd, impl=impl, scratch=scratch)

        h = self._forward(x, pos_tok=xp, slot_tok=xs, attn=attn, k_cache=kc, vt_cache=vc, p0=self.P0, hook=hook)
        # pseudo-row i's copy mask: its state and its input token (the draft before it)
        cm = (self._copy_masks(xst, xt, xs, self.copy_x[off:off + T])
              if sample and self.copy and not (self.sparse and self.argmax) else None)
        if sample and self.argmax:
            # every pseudo-row masked with the state it has if its row's drafts so far are accepted
            best = self.x_best[off:off + T]
            if self.sparse:
                ops.sparse_argmax(h, self.fw_lm, xst, self.fsm, best, xt, xs, self.body_buf, self.body_len,
                                  self.mc.eps)
            else:
                self._argmax(h, xst, best, ss=self._fwd_ss if self.fused else None, row_masks=cm)
            ops.spec_verify_keys(best, self.fsm, self.state[r0:r1], tok, self.out_buf[r0:r1], self.out_len[r0:r1],
                                 done, pos, xt, rs, nd, acc, counts=self.spec_counts)
            logits = best
        else:
            logits = self._logits(h)
        if sample and not self.argmax:
            ops.spec_verify(logits, self.fsm, self.state[r0:r1], tok, self.out_buf[r0:r1], self.out_len[r0:r1], done,
                            pos, xt, rs, nd, acc, row_masks=cm)
        if sample and not self.argmax:
            # tokens emitted and live rows this step (read back only by stats(); the arg-max
            # path adds them inside spec_verify_keys)
            self.spec_counts += torch.stack([acc.sum(dtype=torch.int64), (acc > 0).sum(dtype=torch.int64)])
        return logits

    def reset_stats(self) -> None:
        """Zero the counters (a new measurement window: the idle gap since the last
        chunk is not charged to it)."""
        self.stats.__init__()
        self._idle_prev = None
        self._idle_pairs.clear()

    def spec_stats(self, reset: bool = False) -> Dict[str, float]:
        if not self.spec:
            return {}
        if reset:
            self.spec_counts.zero_()
            return {}
        emitted, live = (int(v) for v in self.spec_counts.tolist())
        return {"spec_tokens": emitted, "spec_row_steps": live,
                "spec_tokens_per_row_step": (emitted / live) if live else 0.0}

    def _side_stream(self) -> torch.cuda.Stream:
        return self._side_streams(1)[0]

    def _side_streams(self, k: int) -> List[torch.cuda.Stream]:
        while len(self._sides) < k:
            self._sides.append(torch.cuda.Stream(device=self.device))
        return self._sides[:k]

    def _decode_steps_split(self, B: int, n: int, s2: torch.cuda.Stream) -> None:
        """``n`` decode steps of rows ``[0, B)`` as two independent half-batches on
        two streams (fork/join), the second half started one QKV GEMM behind the
        first so that one half's memory-bound attention can overlap the other
        half's MFMA GEMMs (nano-batch overlap).  Rows never interact within a
        step, so the result is identical to :meth:`_decode_step` on all rows."""
        h = B // 2
        main = torch.cuda.current_stream(self.device)
        if self.cfg.split_offset:
            # the second half waits for the first half's layer-0 QKV GEMM: from then
            # on half A is in attention while half B runs its GEMMs, and so on
            ev = torch.cuda.Event()
            hook = (lambda i: ev.record() if i == 0 else None)
        else:
            s2.wait_stream(main)
            hook = None
        for k in range(n):
            self._decode_step(h, r0=0, hook=hook if k == 0 else None)
            with torch.cuda.stream(s2):
                if k == 0 and hook is not None:
                    s2.wait_event(ev)
                self._decode_step(B - h, r0=h)
        main.wait_stream(s2)

    # ------------------------------------------------------------ debugging
    def debug_logits(self, bodies: Sequence[str], forced: Sequence[Sequence[int]] = ()) -> List[torch.Tensor]:
        """Logits of the HIP path for validation: the prefill's last position,
        then one decode step per forced token (rows 0..n-1; engine must be idle)."""
        assert not self.active
        items = [_Pending(i, ids) for i, ids in enumerate(self.tok.message_ids(list(bodies), self.cfg.max_body_tokens))]
        n = len(items)
        rows = list(range(n))
        outs = [self._prefill(rows, items, sample=False, templates=False).float()]
        lens = torch.tensor([len(it.ids) for it in items], dtype=torch.int32, device=self.device)
        self.pos[:n] = lens - 1
        self.done[:n] = 0  # attention skips finished rows
        for step in range(len(forced[0]) if forced else 0):
            self.tok_buf[:n] = torch.tensor([f[step] for f in forced], dtype=torch.int32, device=self.device)
            self.pos[:n] += 1
            outs.append(self._decode_step(n, sample=False).float())
        self.done[:n] = 1
        return outs

    def _compact(self) -> None:
        """Move the highest active rows into the lowest free rows when a smaller decode
        bucket would then cover every active row.  Only per-row state moves (token,
        position, FSM state, flags, output buffer); the KV cache stays in its slot —
        rows and slots swap their ``slot_id`` entries.  A row that finished in the
        chunk still in flight is harvested from the next snapshot (done rows stay
        done, their outputs move with them)."""
        if not self.active:
            return
        target = self._bucket(len(self.active))
        if self._bucket(max(self.active) + 1) <= target:
            return
        movers = sorted(r for r in self.active if r >= target)
        free_low = sorted(r for r in self.free_rows if r < target)[: len(movers)]
        if len(free_low) < len(movers):
            return
        dev = self.device
        src = self._stage.to_device(np.asarray(movers, dtype=np.int64), dev)
        dst = self._stage.to_device(np.asarray(free_low, dtype=np.int64), dev)
        for t in (self.tok_buf, self.pos, self.state, self.done, self.out_len, self.out_buf):
            t.index_copy_(0, dst, t.index_select(0, src))
        s_src, s_dst = self.slot_id.index_select(0, src), self.slot_id.index_select(0, dst)
        self.slot_id.index_copy_(0, dst, s_src)
        self.slot_id.index_copy_(0, src, s_dst)
        self.done.index_fill_(0, src, 1)
        self.state.index_fill_(0, src, self.fsm.done_state)
        m, f = np.asarray(movers), np.asarray(free_low)
        self.slot_host[m], self.slot_host[f] = self.slot_host[f].copy(), self.slot_host[m].copy()
        for a, b in zip(movers, free_low):
            self.active[b] = self.active.pop(a)
        taken = set(free_low)
        self.free_rows = [r for r in self.free_rows if r not in taken] + movers
        heapq.heapify(self.free_rows)
        self.stats.compactions += 1
        self.stats.rows_moved += len(movers)

    def _bucket(self, n: int) -> int:
        for b in self.cfg.buckets:
            if b >= n and b <= self.cfg.max_slots:
                return b
        return self.cfg.max_slots

    def _capture_graphs(self) -> None:
        """Capture ``steps_per_graph`` decode steps per bucket (all rows idle/done)."""
        sizes = sorted({self._bucket(b) for b in self.cfg.buckets if b <= self.cfg.max_slots} | {self.cfg.max_slots})
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for B in sizes:  # warm-up: hipBLASLt heuristics/workspaces before capture
                self._decode_step(B)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self._pool = torch.cuda.graph_pool_handle()
        split = self.cfg.split_decode
        s2 = torch.cuda.Stream(device=self.device) if split else None
        parts = max(2, self.cfg.split_parts)
        pools = [self._pool] + [torch.cuda.graph_pool_handle() for _ in range(parts - 1)] \
            if split and self.cfg.split_graphs == 2 else None
        n = self.cfg.steps_per_graph
        for B in sorted(sizes, reverse=True):
            if split and B >= split and pools is not None:
                # one graph per part, replayed concurrently on `parts` streams (_run_decode);
                # one memory pool per part: the parts run at the same time
                bounds = [B * k // parts for k in range(parts + 1)]
                bounds = [b - b % 64 for b in bounds[:-1]] + [B]  # 64-row aligned parts
                bounds = sorted(set(bounds))  # a bucket too small for `parts` gets fewer
                gs = []
                for k in range(len(bounds) - 1):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=pools[k]):
                        for _ in range(n):
                            self._decode_step(bounds[k + 1] - bounds[k], r0=bounds[k])
                    gs.append(g)
                self.graphs[B] = tuple(gs) if len(gs) > 1 else gs[0]
                continue
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self._pool):
                if split and B >= split:
                    self._decode_steps_split(B, n, s2)
                else:
                    for _ in range(n):
                        self._decode_step(B)
            self.graphs[B] = g
        torch.cuda.synchronize(self.device)

    def _run_decode(self, B: int) -> None:
        t0 = time.perf_counter()
        g = self.graphs.get(B)
        if isinstance(g, tuple):
            main = torch.cuda.current_stream(self.device)
            sides = self._side_streams(len(g) - 1)
            for s in sides:
                s.wait_stream(main)
            g[0].replay()
            for s, gk in zip(sides, g[1:]):
                with torch.cuda.stream(s):
                    gk.replay()
            for s in sides:
                main.wait_stream(s)
            n = self.cfg.steps_per_graph
        elif g is not None:
            g.replay()
            n = self.cfg.steps_per_graph
        else:
            self._decode_step(B)
            n = 1
        self.stats.decode_steps += n
        self.stats.decode_row_steps += n * B
        self.stats.decode_s += time.perf_counter() - t0

    # -------------------------------------------------------------- scheduler
    def submit(self, key: Any, body: str) -> None:
        ids = self.tok.message_ids([body], self.cfg.max_body_tokens)[0]
        self.waiting.append(_Pending(key, ids))

    def submit_many(self, items: Sequence[Tuple[Any, str]]) -> None:
        if not items:
            return
        enc = self.tok.message_ids([b for _, b in items], self.cfg.max_body_tokens)
        for (k, _), ids in zip(items, enc):
            self.waiting.append(_Pending(k, ids))

    def busy(self) -> bool:
        return bool(self.waiting or self.active or self._pending is not None)

    def _admit(self) -> None:
        S = self.cfg.max_slots
        if not self.waiting or not self.free_rows:
            return
        if self.active and len(self.free_rows) < max(1, int(S * self.cfg.admit_min_fraction)) \
                and len(self.free_rows) < len(self.waiting):
            return
        if (self.active and len(self.waiting) < self.cfg.admit_min_batch
                and time.perf_counter() - self.waiting[0].t < self.cfg.admit_max_wait_s):
            return
        while self.waiting and self.free_rows:
            rows, items, ntok = [], [], 0
            while self.waiting and self.free_rows:
                it = self.waiting[0]
                if items and ntok + len(it.ids) > self.cfg.prefill_max_tokens:
                    break
                self.waiting.popleft()
                r = heapq.heappop(self.free_rows)
                rows.append(r)
                items.append(it)
                ntok += len(it.ids)
                self.active[r] = it.key
            self._learn_templates(items)
            split = self.cfg.split_prefill
            if split and ntok >= split and len(items) >= 2:
                # two independent halves on two streams (disjoint rows and KV slots):
                # one half's latency-bound attention overlaps the other's GEMMs
                h = len(items) // 2
                main = torch.cuda.current_stream(self.device)
                s2 = self._side_stream()
                s2.wait_stream(main)
                self._prefill(rows[:h], items[:h])
                with torch.cuda.stream(s2):
                    self._prefill(rows[h:], items[h:])
                main.wait_stream(s2)
            else:
                self._prefill(rows, items)

    def _decode_answer(self, toks: List[int]) -> Dict[str, Optional[str]]:
        vals = self.fsm.split_fields(toks)
        out: Dict[str, Optional[str]] = {}
        for i, f in enumerate(self.fsm.fields):
            out[f.name] = self.tok.decode(vals[i]).strip() if i < len(vals) else None
        return out

    def _snapshot(self, B: int) -> "_Snapshot":
        """Queue an async D2H copy of the row state after the chunk just launched."""
        i = self._snap_flip
        self._snap_flip ^= 1
        hb = self._host_bufs[i]
        hb["done"][:B].copy_(self.done[:B], non_blocking=True)
        hb["len"][:B].copy_(self.out_len[:B], non_blocking=True)
        hb["buf"][:B].copy_(self.out_buf[:B], non_blocking=True)
        # a blocking-sync event: the harvest's wait for the chunk sleeps instead of spinning
        # a core (the rank process spent ~45 % of its CPU time spinning in this wait)
        ev = torch.cuda.Event(enable_timing=self.cfg.measure_idle, blocking=True)
        ev.record()
        return _Snapshot(B, ev, hb, dict(self.active))

    def _harvest(self, snap: "_Snapshot", raw: bool = False) -> List[Tuple[Any, Any]]:
        t0 = time.perf_counter()
        snap.event.synchronize()
        self.stats.harvest_wait_s += time.perf_counter() - t0
        done_h = snap.bufs["done"][: snap.B].numpy()
        res: List[Tuple[Any, Any]] = []
        lens = snap.bufs["len"]
        bufs = snap.bufs["buf"]
        fin = [r for r, key in snap.active.items()
               if r < snap.B and done_h[r] and self.active.get(r) is key]
        if fin and raw:
            # token ids only (a remote client detokenises): one gather copy of the finished
            # rows out of the reused pinned snapshot, then per-row views of it
            lens_l = lens.numpy()[fin].tolist()
            blk = bufs.numpy()[fin]
            active, free = self.active, self.free_rows
            for j, r in enumerate(fin):
                res.append((active.pop(r), blk[j, : lens_l[j]]))
                heapq.heappush(free, r)
        elif fin:
            # one batched detokenisation (Rust, parallel) for every field of every finished row
            nf = len(self.fsm.fields)
            lens_l = lens[fin].tolist()
            rows_l = bufs[fin].tolist()
            pieces: List[List[int]] = []
            for toks, n in zip(rows_l, lens_l):
                vals = self.fsm.split_fields(toks[:n])
                vals += [[]] * (nf - len(vals))
                pieces.extend(vals)
            texts = self.tok.decode_batch(pieces)
            for j, r in enumerate(fin):
                ans = null_rejection({f.name: texts[j * nf + i].strip() for i, f in enumerate(self.fsm.fields)})
                res.append((self.active.pop(r), ans))
                heapq.heappush(self.free_rows, r)
        self.stats.completed += len(res)
        self.stats.harvest_s += time.perf_counter() - t0
        return res

    def step(self, raw: bool = False) -> List[Tuple[Any, Any]]:
        """Admit → launch one decode chunk → harvest the *previous* chunk's snapshot
        (the GPU runs chunk k while the host decodes chunk k-1's finished rows).
        Admitting first lets new rows join the very next chunk: launching the chunk
        before the admission's host prep was measured slower (one more chunk of
        padded rows per admission outweighs the hidden prep).  Returns finished
        ``(key, answer dict)`` — or ``(key, int32 token array)`` with ``raw=True``
        (the remote-client path)."""
        t0 = time.perf_counter()
        if self.cfg.measure_idle and self._idle_prev is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()  # runs when the GPU reaches this step's first work
            self._idle_pairs.append((self._idle_prev, ev))
            self._idle_prev = None
        if self.cfg.compact:
            self._compact()
        t1 = time.perf_counter()
        self._admit()
        self.stats.compact_s += t1 - t0
        self.stats.admit_s += time.perf_counter() - t1
        prev, self._pending = self._pending, None
        if self.active:
            B = self._bucket(max(self.active) + 1)
            self._run_decode(B)
            self._pending = self._snapshot(B)
            if self.cfg.measure_idle:
                self._idle_prev = self._pending.event
        out = self._harvest(prev, raw) if prev is not None else []
        while self._idle_pairs and self._idle_pairs[0][1].query():
            a, b = self._idle_pairs.popleft()
            self.stats.gpu_idle_s += max(0.0, a.elapsed_time(b)) / 1000.0
        self.stats.steps += 1
        self.stats.step_s += time.perf_counter() - t0
        return out

    def submit_ids(self, items: Sequence[Tuple[Any, Sequence[int]]]) -> None:
        """Queue pre-tokenised prompts (``body <ans>`` ids, see the tokenizer)."""
        cap = self.cfg.max_body_tokens + 2
        for k, ids in items:
            if len(ids) > cap:  # keep the closing <ans>
                ids = np.concatenate([np.asarray(ids[: cap - 1], dtype=np.int32), np.asarray(ids[-1:], dtype=np.int32)])
            self.waiting.append(_Pending(k, ids))

    def run(self, bodies: Sequence[str]) -> List[Dict[str, Optional[str]]]:
        """Synchronous batch extraction (tests, benchmarks)."""
        self.submit_many(list(enumerate(bodies)))
        out: List[Optional[Dict[str, Optional[str]]]] = [None] * len(bodies)
        while self.busy():
            for k, ans in self.step():
                out[k] = ans
        return out  # type: ignore[return-value]
