"""``local_llm`` backend: the extraction LM served on this process's MI355X.

Replaces the remote ``call_gemini`` (gemini_parser.py:273-292) behind the same
boundary.  Answers have the Gemini JSON shape (nine string fields) so the
post-processing chain is unchanged.  One backend instance = one GPU = one
engine thread; under ``torchrun`` every rank builds its own (data-parallel
replicas consuming ``sms.raw`` as one competing consumer group —
:mod:`smsgate_amd.parallel`).

Weights: ``LLM_CHECKPOINT`` (safetensors, serving layout), else the trained
checkpoint bundled for ``LLM_MODEL`` if there is one.  With neither,
:func:`build_engine` **refuses to start** (:class:`MissingCheckpoint`):
random-init output is schema-valid but meaningless, so a silent fallback would
route every SMS to the DLQ.  Random weights are only for throughput runs and
must be asked for (``random_init=True``, ``engine-server --random-init``).
"""
from __future__ import annotations

import os
from typing import Any, List, Optional, Sequence

from ...runtime.errors import TransientError
from .base import BackendError, ExtractResult, ParserBackend

__all__ = ["LocalLLMBackend", "RemoteLLMBackend", "build_engine", "MissingCheckpoint", "resolve_checkpoint"]


class MissingCheckpoint(RuntimeError):
    """No trained weights for the requested model and random init not requested."""


def bundled_checkpoint(model: str) -> Optional[str]:
    """A trained checkpoint shipped with the package (``models/assets/extractor-<model>.safetensors``;
    produced by ``python -m smsgate_amd train-extractor``), or None."""
    from pathlib import Path

    p = Path(__file__).resolve().parents[2] / "models" / "assets" / f"extractor-{model}.safetensors"
    return str(p) if p.exists() else None


def resolve_checkpoint(model: str, checkpoint: Optional[str] = None, random_init: bool = False) -> Optional[str]:
    """The weights file to serve: ``checkpoint``, else ``LLM_CHECKPOINT``, else the
    bundled checkpoint of ``model``; None only with ``random_init``.  Raises
    :class:`MissingCheckpoint` otherwise (and when a named file does not exist)."""
    if random_init:
        return None
    ck = checkpoint or os.getenv("LLM_CHECKPOINT") or bundled_checkpoint(model)
    if not ck:
        raise MissingCheckpoint(
            f"no trained checkpoint for model {model!r}: set LLM_CHECKPOINT / --checkpoint to a safetensors file "
            f"(python -m smsgate_amd train-extractor --model {model} --out ...), or pass --random-init for a "
            "throughput-only run")
    if not os.path.exists(ck):
        raise MissingCheckpoint(f"checkpoint {ck!r} does not exist")
    return ck


def build_engine(model: str = "smollm-135m", checkpoint: Optional[str] = None, device: str = "cuda",
                 seed: int = 0, random_init: bool = False, weights=None, answer_format: str = "qa",
                 **engine_kw: Any):
    """Engine for ``model`` with the weights :func:`resolve_checkpoint` picks;
    ``random_init=True`` serves random weights (throughput benchmarks only; in
    ``answer_format`` "span" they are a span-pointer model's); ``weights`` serves an
    in-memory :class:`ExtractorWeights` (e.g. just trained).  A checkpoint's answer
    format comes from its own metadata; ``answer_format`` (default "qa", the flagship
    one-forward head) only shapes random-init weights."""
    import torch

    from ...models.extractor import CONFIGS, ExtractorWeights, qa_config, span_config
    from ...models.tokenizer import load_tokenizer
    from ...serving.engine import EngineConfig, ExtractionEngine
    from ...serving.qa_engine import QAEngine

    if answer_format == "span":
        cfg = span_config(CONFIGS[model])
    elif answer_format in ("qa", "qa17"):
        cfg = qa_config(CONFIGS[model], queries=9 if answer_format == "qa" else 17)
    elif answer_format == "copy":
        cfg = CONFIGS[model]
    else:
        raise ValueError(f"answer format {answer_format!r}: copy | span | qa | qa17")

    def make(w):
        # the weights' own format picks the engine: one forward (qa) or pointer decode
        cls = QAEngine if w.cfg.qa_queries > 0 else ExtractionEngine
        return cls(w, load_tokenizer(), EngineConfig(**engine_kw))

    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if weights is not None:
        weights.requires_grad_(False)
        return make(weights)
    checkpoint = resolve_checkpoint(model, checkpoint, random_init)
    if checkpoint:
        w = ExtractorWeights.load(checkpoint, cfg, device=dev)
    else:
        w = ExtractorWeights(cfg, device=dev, seed=seed)
    w.requires_grad_(False)
    return make(w)


class LocalLLMBackend(ParserBackend):
    name = "local_llm"

    def __init__(self, model: Optional[str] = None, checkpoint: Optional[str] = None, device: Optional[str] = None,
                 max_slots: int = 1024, max_batch: Optional[int] = None, **engine_kw: Any) -> None:
        self.model = model or os.getenv("LLM_MODEL", "smollm-135m")
        self.checkpoint = checkpoint or os.getenv("LLM_CHECKPOINT") or None
        self.device = device or os.getenv("LLM_DEVICE", "cuda")
        self.engine_kw = dict(max_slots=max_slots, **engine_kw)
        self.max_batch = max_batch or max_slots
        self._worker = None
        self._factory = None

    @classmethod
    def from_engine(cls, engine, max_batch: Optional[int] = None) -> "LocalLLMBackend":
        """Serve an already-built :class:`~smsgate_amd.serving.engine.ExtractionEngine`
        (e.g. freshly trained weights) through the backend interface."""
        be = cls(max_slots=engine.cfg.max_slots, max_batch=max_batch)
        be._factory = lambda: engine
        return be

    async def start(self) -> None:
        if self._worker is not None:
            return
        import asyncio

        from ...serving.worker import EngineWorker

        w = EngineWorker(self._factory or (lambda: build_engine(self.model, self.checkpoint, self.device,
                                                                **self.engine_kw)))
        await asyncio.to_thread(w.start)
        self._worker = w

    async def close(self) -> None:
        if self._worker is not None:
            import asyncio

            await asyncio.to_thread(self._worker.stop)
            self._worker = None

    @property
    def engine(self):
        return None if self._worker is None else self._worker.engine

    async def extract_batch(self, bodies: Sequence[str]) -> List[ExtractResult]:
        if self._worker is None:
            await self.start()
        res = await self._worker.extract(bodies)  # type: ignore[union-attr]
        out: List[ExtractResult] = []
        for r in res:
            if isinstance(r, BaseException):
                out.append(r)
            elif r is None:
                out.append(BackendError("local LLM produced no answer"))
            else:
                out.append(dict(r))
        return out


class RemoteLLMBackend(ParserBackend):
    """The same extractor, served by an engine process on the GPU
    (:class:`~smsgate_amd.serving.remote.EngineServer`); this process only
    tokenises, ships ids and detokenises — the multi-process replica layout."""

    name = "local_llm"

    def __init__(self, client, max_batch: int = 512) -> None:
        self.client = client
        self.max_batch = max_batch

    async def extract_batch(self, bodies: Sequence[str]) -> List[ExtractResult]:
        try:
            return list(await self.client.extract(bodies))
        except TransientError:
            raise  # engine unreachable: the stage naks the batch (no DLQ traffic)
        except Exception as exc:  # noqa: BLE001 — every message of the batch fails loudly
            return [exc] * len(bodies)

    async def extract_rows(self, bodies: Sequence[str]) -> List[Any]:
        """:meth:`extract_batch` as the nine decoded field strings per answer (no dicts:
        the pipeline's native post-processing reads them, parse/fastpath.py); the same
        failure semantics."""
        try:
            return list(await self.client.extract_rows(bodies))
        except TransientError:
            raise
        except Exception as exc:  # noqa: BLE001
            return [exc] * len(bodies)
