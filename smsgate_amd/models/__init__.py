"""Model families of the framework.

* :mod:`.domain` — the wire schema (RawSMS / ParsedSMS / ParsedSmsCore).
* :mod:`.extractor` — the local structured-extraction decoder LM run on MI355X
  (imported lazily: it needs torch).
* :mod:`.tokenizer` — byte-level BPE tokenizer for the extractor.
"""
from .domain import (  # noqa: F401
    CORE_FIELDS,
    PARSER_VERSION_LLM,
    ParsedSMS,
    ParsedSmsCore,
    RawSMS,
    TxnType,
    get_md5_hash,
    get_sha1_hash,
)
