"""The pipeline's services (each one a process in production, or all in one).

=================  ================================================  ==========================
module             role                                              reference
=================  ================================================  ==========================
``gateway``        FastAPI ``POST /sms/raw``, ``/health``, metrics   services/api_gateway
``parser``         ``sms.raw`` → parse → ``sms.parsed``/DLQ          services/parser_worker
``writer``         ``sms.parsed`` → PocketBase + SQL                 services/pb_writer
``dlq``            ``sms.failed`` inspector / re-parser              parser_worker/dlq_worker
``xml_watcher``    XML backup directory poller                       services/xml_watcher
``notifier``       PocketBase → chart → Telegram                     services/dashboard
``mcp_server``     SQL tools over MCP (JSON-RPC / SSE)               services/mcp_server
``receiver``       webhook capture server                            receiver.py
``legacy``         cache loaders / batch re-processing tools         read_xml.py, process_cached.py, …
=================  ================================================  ==========================
"""
