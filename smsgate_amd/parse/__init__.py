"""SMS parse pipeline (the reference's ``libs/gemini_parser.py`` + helpers)."""
from .dates import fix_broken_datetime, parse_custom_datetime, parse_unix_timestamp  # noqa: F401
from .numeric import parse_ambiguous_decimal  # noqa: F401
from .pipeline import BrokenMessage, Outcome, ParsePipeline, ParseResult, postprocess_answer  # noqa: F401
from .text import (  # noqa: F401
    extract_json,
    llm_should_skip,
    mask_card_number_with_prefix,
    normalize_body,
    worker_should_skip,
)
