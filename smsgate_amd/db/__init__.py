"""Persistence schema and migrations (reference ``db/``)."""
from .schema import metadata, parsed_to_row, sms_data  # noqa: F401
