"""The benchmark harness through ONE shared native broker: two ranks (gloo, CPU echo
engines) whose parser and writer processes form single competing groups on one
smsgate-busd; every message is routed once and written once."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "smsgate_amd/native/_bin/smsgate-busd")),
                    reason="native broker not built")
def test_two_ranks_one_broker():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29671", "bench.py", "--gpus", "2", "--cpu-echo-engine",
           "--steps", "2", "--warmup", "1", "--msgs-per-step", "1024", "--cpu-workers", "2", "--bus", "busd"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert r.returncode == 0 and len(lines) == 1, r.stderr[-3000:]
    out = lines[0]
    rt = out["routing"]
    total = 2 * 2 * 1024  # ranks x steps x msgs per step
    assert rt["parsed"] + rt["keyword_skipped"] + rt["broken"] + rt["dlq"] == total
    assert rt["sink_stored"] + rt["writer_no_merchant"] == rt["parsed"]  # every parsed message written once
    assert "shared smsgate-busd" in out["config"]["bus"] and out["n_gpus"] == 2
    # node CPU budget of the timed region: every role accounted, brokers included
    cpu = out["cpu"]
    assert set(cpu["cores_busy_per_gpu"]) == {"parser_procs", "rank_proc", "brokers"}
    # the HTTP-ingest phase: loaders POST every SMS to the native doors; their CPU is client-side
    h = out["http_ingest"]
    assert h["endpoint"] == "/sms/raw" and h["requests"] == total and h["value"] > 0
    assert h["cpu"].get("client_loaders", {"cpu_us_per_msg": 1})["cpu_us_per_msg"] > 0
    assert cpu["cores_busy_per_gpu"]["parser_procs"] > 0 and cpu["cores_busy_per_gpu"]["brokers"] > 0
    assert cpu["cpu_us_per_msg"] > 0 and abs(cpu["node_cores_at_8_gpus"] - 8 * cpu["cores_busy_per_gpu_total"]) <= 0.1  # (from unrounded)
    assert not [d for d in os.listdir("/tmp") if d == "smsgate-bench-bus-29671"]  # broker dir cleaned up


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "smsgate_amd/native/_bin/smsgate-busd")),
                    reason="native broker not built")
def test_bench_with_a_real_sql_sink():
    """--sink sqlite: every parser process's writer upserts into its own SQLite WAL file
    (SqlSink) inside the timed region; every parsed message is stored once."""
    cmd = [sys.executable, "bench.py", "--cpu-echo-engine", "--steps", "2", "--warmup", "1", "--msgs-per-step", "1024",
           "--cpu-workers", "2", "--bus", "busd", "--sink", "sqlite"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert r.returncode == 0 and len(lines) == 1, r.stderr[-3000:]
    rt = lines[0]["routing"]
    assert rt["sink_stored"] + rt["writer_no_merchant"] == rt["parsed"] > 0 and rt["writer_fail"] == 0
    assert not [d for d in os.listdir("/tmp") if d.startswith("smsgate-bench-sink-r0-")]  # sink files removed


def test_stale_broker_socket_is_not_listening(tmp_path):
    """A socket file whose broker died (a crashed run with the same MASTER_PORT) does not
    count as the node broker: the waiting ranks hold until a live one accepts."""
    import socket

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    path = str(tmp_path / "bus0.sock")
    assert not bench._listening(path)
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(path)
    srv.listen(1)
    assert bench._listening(path)
    srv.close()  # the file stays, nobody accepts
    assert os.path.exists(path) and not bench._listening(path)


@pytest.mark.slow
@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "smsgate_amd/native/_bin/smsgate-busd")),
                    reason="native broker not built")
def test_eight_ranks_full_node_layout():
    """VERDICT r03 next #4b / r04 next #3: 8 ranks (gloo, CPU echo engines) through the
    production node layout (bus/sharded.py NODE_PARTITIONS: sms.raw, sms.parsed and
    sms.processing partitioned, one broker for the rest) with one parser process each:
    exact routing totals, traffic on every partition of every partitioned subject, and a
    drain that accounts for every message across the raw partitions."""
    from smsgate_amd.bus.sharded import NODE_PARTITIONS

    ranks, steps, warm, per = 8, 2, 1, 512
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
           "--master-addr", "127.0.0.1", "--master-port", "29683", "bench.py", "--gpus", str(ranks),
           "--cpu-echo-engine", "--steps", str(steps), "--warmup", str(warm), "--msgs-per-step", str(per),
           "--cpu-workers", "1", "--bus", "busd", "--rank-threads", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900, env=env)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert r.returncode == 0 and len(lines) == 1, r.stderr[-3000:]
    out = lines[0]
    rt = out["routing"]
    total = ranks * steps * per
    assert out["n_gpus"] == ranks and rt["parsed"] + rt["keyword_skipped"] + rt["broken"] + rt["dlq"] == total
    assert rt["sink_stored"] + rt["writer_no_merchant"] == rt["parsed"], json.dumps(rt)
    for subj, n in NODE_PARTITIONS.items():
        assert f"{subj} over {n}" in out["config"]["bus"], out["config"]["bus"]
    members = out["bus_members"]
    assert len(members) == sum(NODE_PARTITIONS.values()) + 1
    by = {subj: [m for m in members if m["subjects"] == [subj]] for subj in NODE_PARTITIONS}
    assert {s: len(v) for s, v in by.items()} == NODE_PARTITIONS
    raw = by["sms.raw"]
    # every raw message of the run stored on exactly one raw partition: the bus-ingest
    # phase (warmup + steps) and the HTTP-ingest phase (1 warmup step + steps) through
    # the raw partitions' native /sms/raw doors
    assert sum(m["messages"] for m in raw) == ranks * (steps + warm) * per + ranks * (steps + 1) * per
    assert all(m["messages"] > 0 for v in by.values() for m in v), str([(m["subjects"][0][4:], m["messages"]) for m in members])
    # the parser's two outputs per parsed SMS land on their own partitions, evenly
    for subj in ("sms.parsed", "sms.processing"):
        counts = [m["messages"] for m in by[subj]]
        assert max(counts) <= 1.5 * min(counts) + 64, (subj, counts)
    h = out["http_ingest"]
    assert h["requests"] == total and h["routing"]["parsed"] + h["routing"]["keyword_skipped"] + \
        h["routing"]["broken"] + h["routing"]["dlq"] == total
