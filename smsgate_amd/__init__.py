"""smsgate_amd — an MI355X-native SMS-to-transaction pipeline framework.

Capability parity with vpuhoff/smsgate (reference snapshot 2025-09-05):

* HTTP ingestion (``POST /sms/raw``) and XML-backup ingestion,
* a durable subject bus with durable consumer groups, explicit ack/nak,
  ack-wait redelivery, max-age retention and a dead-letter subject,
* an LLM parse pipeline (pre-filter → normalise → cache → extract →
  post-process → validate) behind a pluggable :class:`ParserBackend`,
* idempotent persistence (SQL ``ON CONFLICT(msg_id)``, PocketBase REST),
* Prometheus metrics, Sentry-style error capture and tracing spans,
* a Telegram summary notifier and MCP query tools.

The MI355X-first part is the ``local_llm`` parser backend: a
schema-constrained extraction LM served with hand-written HIP/CDNA4 kernels
(``smsgate_amd.ops``), continuous batching with HIP-graph-captured decode
steps (``smsgate_amd.serving``), and one data-parallel replica per GPU
(``smsgate_amd.parallel``) acting as competing consumers on ``sms.raw``.
"""

__version__ = "0.1.0"

__all__ = ["__version__"]
