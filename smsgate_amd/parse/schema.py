"""The extraction contract shared by every parser backend.

* :data:`CORE_FIELDS` — the nine keys, in schema order (llm_core.py:9-19).
* :data:`SYSTEM_INSTRUCTION` — the system prompt sent with every extraction
  request; same content and key list as the reference's Gemini prompt
  (gemini_parser.py:37-43) so remote and local backends see one task.
* :data:`EXTRACTOR_PROMPT` — the local extractor's prompt.  The extractor is
  trained on the task, so the instruction lives in its weights and the prompt is
  a two-token task tag (a 242-token Russian instruction would be 60 % of every
  training sequence and of every decode step's attention for no information: it
  is constant).  Round 3 cut the tag from the schema key list (``<bos> Extract:
  txn_type date … <sms>``, 21 shared keys) to ``<bos> txn: <sms>`` (4 keys): every
  decode and prefill query attends to the shared keys, and with 4 of them
  (a multiple of 4) the attention kernels walk them inside the row's own key
  stream (``ops.set_attn_merge``) instead of a padded 32-key tile of their own.
* :data:`RESPONSE_SCHEMA` — the JSON schema of the answer: nine string
  properties, ``txn_type`` and ``date`` required (gemini_parser.py:46-61),
  expressed as plain JSON (the REST API shape), not google-genai objects.
* :data:`TXN_TYPES` — the enum values a constrained decoder may emit.
"""
from __future__ import annotations

from ..models.domain import CORE_FIELDS, TxnType

__all__ = ["CORE_FIELDS", "SYSTEM_INSTRUCTION", "EXTRACTOR_PROMPT", "RESPONSE_SCHEMA", "TXN_TYPES",
           "GENERATION_TEMPERATURE"]

TXN_TYPES = tuple(t.value for t in TxnType)

GENERATION_TEMPERATURE = 0.1  # gemini_parser.py:216

SYSTEM_INSTRUCTION = (
    "Ты — банковский парсер. Верни ТОЛЬКО JSON "
    f"со строго следующими ключами: {', '.join(CORE_FIELDS)}. "
    "Без Markdown-обёрток и лишнего текста."
    "txn_type может иметь значения 'debit', 'credit', 'otp' или 'unknown'"
    "Дата в сообщении обычно в формате день.месяц.год часы:минуты"
)

EXTRACTOR_PROMPT = "txn:"

RESPONSE_SCHEMA = {
    "type": "OBJECT",
    "properties": {name: {"type": "STRING"} for name in CORE_FIELDS},
    "required": ["txn_type", "date"],
}
