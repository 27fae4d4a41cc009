"""Error classes the consume loop (:mod:`smsgate_amd.runtime.stage`) routes on."""
from __future__ import annotations

__all__ = ["TransientError"]


class TransientError(Exception):
    """A failure of a dependency, not of the message (an engine restart, a broken
    socket).  A handler raising it gets its whole batch nak'ed with backoff; the
    batch is not split to hunt for a poison message and no delivery counts
    towards dead-lettering."""
