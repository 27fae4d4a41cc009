"""GPU serving runtime of the local extractor: schema FSM, engine, worker thread."""
from .fsm import DEFAULT_FIELDS, FieldSpec, SchemaFSM, build_fsm  # noqa: F401
