"""Broker capacity for an 8-GPU node.

A node of 8 GPUs at the headline rate (~21 k SMS/s each) needs, per SMS, one
sms.raw publish + delivery + ack (ingest -> parser) and two publishes plus one
delivery + ack on the parser's outputs (sms.parsed / sms.processing -> writer).
The benchmark runs two ``smsgate-busd`` brokers sharded by subject
(:mod:`smsgate_amd.bus.sharded`).  Here both run with their journals on (fsync
interval, as deployed) under the native load generator with 64 competing
consumers in total, and together must sustain >= 3 x (8 x the headline)
publish -> fetch -> ack messages per second.
"""
import json
import subprocess

import pytest

from smsgate_amd.native import BUSD, available, spawn_busd
from smsgate_amd.native.build import BUSLOAD

HEADLINE_PER_GPU = 21_000  # msgs/s on one MI355X (profiles/r02_bus_spec_ab.jsonl)
TARGET = 3 * 8 * HEADLINE_PER_GPU


@pytest.mark.skipif(not (available(BUSD) and BUSLOAD.exists()), reason="native broker / load generator not built")
def test_two_sharded_brokers_carry_an_8_gpu_node(tmp_path):
    best = 0.0
    for attempt in range(2):  # best of two: the load generators share the CPUs with the brokers
        socks = [tmp_path / f"a{attempt}.sock", tmp_path / f"b{attempt}.sock"]
        brokers = [spawn_busd(f"unix://{s}", str(tmp_path / f"data{attempt}{k}")) for k, s in enumerate(socks)]
        try:
            procs = [subprocess.Popen([str(BUSLOAD), "--socket", str(s), "--producers", "2", "--consumers", "32",
                                       "--msgs", "200000"], stdout=subprocess.PIPE, text=True) for s in socks]
            outs = [json.loads(p.communicate(timeout=120)[0]) for p in procs]
        finally:
            for b in brokers:
                b.stop()
        assert all(o["ok"] and o["acked"] >= o["published"] == 400000 for o in outs), outs
        best = max(best, sum(o["publish_per_s"] for o in outs))
        if best >= TARGET:
            break
    assert best >= TARGET, f"{best:.0f} msgs/s < {TARGET}"
