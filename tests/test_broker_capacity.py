"""Broker capacity for an 8-GPU node.

A node of 8 GPUs at the headline rate moves one message per SMS on each per-SMS
subject: sms.raw (ingest -> parser: publish + delivery + ack), sms.parsed (parser ->
writer) and sms.processing (parser -> downstream: published per parsed SMS), plus the
DLQ traffic on the rest broker.  The node layout (bus/sharded.py NODE_PARTITIONS,
deploy/docker-compose.yml generated from it) partitions the three per-SMS subjects,
so EVERY broker carries ``8 x headline x share(subject) / partitions`` messages per
second, ``share`` measured per member (``bus_members`` of the newest committed bench
line, profiles/r*_bench*.json: each member's messages over the sms.raw messages) and
the headline the latest driver-measured BENCH (``BENCH_r*.json``), not a constant.

One broker, journal on (fsync interval, as deployed), under the native load generator
with 16 competing consumers, must sustain TWICE the most loaded member's need (best of
three: the load generator shares this box's 8 vCPUs with the broker); the raw
partitions' native HTTP doors, at their measured single-SMS request rate, twice the
node rate.
"""
import glob
import json
import os
import re
import subprocess

import pytest

from smsgate_amd.bus import SUBJECT_PARSED, SUBJECT_PROCESSING, SUBJECT_RAW
from smsgate_amd.bus.sharded import NODE_PARTITIONS, Router, node_layout, parse_members
from smsgate_amd.native import BUSD, available, spawn_busd
from smsgate_amd.native.build import BUSLOAD

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADROOM = 2.0
GPUS_PER_NODE = 8


def latest_headline() -> float:
    """msgs/s of the newest driver BENCH record (one MI355X)."""
    best = None
    for p in glob.glob(os.path.join(ROOT, "BENCH_r*.json")):
        m = re.search(r"BENCH_r(\d+)\.json$", p)
        rec = json.load(open(p))
        val = (rec.get("parsed") or {}).get("value")
        if m and val:
            if best is None or int(m.group(1)) > best[0]:
                best = (int(m.group(1)), float(val))
    assert best is not None, "no BENCH_r*.json with a value"
    return best[1]


def measured_shares():
    """Per-SMS message share of each subject of the layout and of the rest broker, from
    the newest committed bench line with ``bus_members`` (None: no such line)."""
    best = None
    for p in glob.glob(os.path.join(ROOT, "profiles", "r*_bench*.json")):
        try:
            rec = json.loads([x for x in open(p) if x.startswith("{")][-1])
        except (ValueError, IndexError):
            continue
        if str(rec.get("weights", "")).startswith("random"):
            continue  # random weights dead-letter every message: not the traffic mix
        if rec.get("bus_members") and all("messages" in m for m in rec["bus_members"]):
            key = (os.path.basename(p)[:3], os.path.getmtime(p))
            if best is None or key > best[0]:
                best = (key, rec["bus_members"])
    if best is None:
        return None
    members = best[1]
    raw = sum(m["messages"] for m in members if m["subjects"] == [SUBJECT_RAW])
    out = {}
    for m in members:
        subj = m["subjects"][0] if len(m["subjects"]) == 1 else "*"
        out[subj] = out.get(subj, 0) + m["messages"] / max(1, raw)
    if SUBJECT_PROCESSING not in out and SUBJECT_PARSED in out:
        # a run of the older layout: its rest broker also carried sms.processing (one
        # publish per parsed SMS, like sms.parsed)
        out[SUBJECT_PROCESSING] = out[SUBJECT_PARSED]
        out["*"] = max(0.0, out.get("*", 0.0) - out[SUBJECT_PARSED])
    return out


def member_needs():
    """msgs/s each member of the 8-GPU node layout carries at the latest headline:
    {member label: need}.  Shares default to 1 per per-SMS subject and 1 for the rest
    broker (every message dead-lettered) when no measured split exists."""
    node = GPUS_PER_NODE * latest_headline()
    shares = measured_shares() or {}
    needs = {}
    for subj, n in NODE_PARTITIONS.items():
        for k in range(n):
            needs[f"{subj}#{k}"] = node * shares.get(subj, 1.0) / n
    needs["*"] = node * shares.get("*", 1.0)
    return needs


def test_every_member_is_sized():
    needs = member_needs()
    assert len(needs) == sum(NODE_PARTITIONS.values()) + 1
    node = GPUS_PER_NODE * latest_headline()
    # no broker carries more than half of any per-SMS subject's node rate
    for subj, n in NODE_PARTITIONS.items():
        assert n >= 2 and max(v for k, v in needs.items() if k.startswith(subj + "#")) <= 0.5 * node * 1.05


@pytest.mark.skipif(not (available(BUSD) and BUSLOAD.exists()), reason="native broker / load generator not built")
def test_one_broker_carries_twice_the_busiest_members_share(tmp_path):
    target = HEADROOM * max(member_needs().values())
    best = 0.0
    for attempt in range(3):  # best of three: the load generator shares the CPUs with the broker
        sock = tmp_path / f"b{attempt}.sock"
        broker = spawn_busd(f"unix://{sock}", str(tmp_path / f"data{attempt}"))
        try:
            p = subprocess.Popen([str(BUSLOAD), "--socket", str(sock), "--producers", "2", "--consumers", "16",
                                  "--msgs", "200000"], stdout=subprocess.PIPE, text=True)
            out = json.loads(p.communicate(timeout=120)[0])
        finally:
            broker.stop()
        assert out["ok"] and out["acked"] >= out["published"] == 400000, out
        best = max(best, out["publish_per_s"])
        if best >= target:
            break
    assert best >= target, f"{best:.0f} msgs/s < {target:.0f} (2 x the busiest member's need)"


def test_ingest_doors_have_twice_the_node_rate():
    """The sms.raw partitions' native HTTP doors (one per raw broker), at their measured
    single-SMS request rate (median of profiles/r03_ingest_bench.jsonl), take twice the
    node rate of one-SMS POSTs (the reference's api_gateway contract)."""
    recs = [json.loads(x) for x in open(os.path.join(ROOT, "profiles", "r03_ingest_bench.jsonl"))]
    native = sorted(r["single"]["requests_per_s"] for r in recs if r["mode"] == "native" and r.get("lossless"))
    per_door = native[len(native) // 2]
    node = GPUS_PER_NODE * latest_headline()
    assert NODE_PARTITIONS[SUBJECT_RAW] * per_door >= HEADROOM * node, (NODE_PARTITIONS[SUBJECT_RAW], per_door, node)
