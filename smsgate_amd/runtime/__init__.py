"""Service runtime: the batch consume loop, retries, process lifecycle."""
from .retry import RetryError, retry  # noqa: F401
from .stage import Stage  # noqa: F401
