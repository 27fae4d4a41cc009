"""The measurement helpers whose numbers the docs quote: GPU time per message from
rocprofv3 kernel stats (CSV or the SQLite output), and the cProfile top-N summary."""
import csv
import json
import sqlite3
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _bench_line(path: Path) -> None:
    path.write_text("noise\n" + json.dumps({"value": 1000.0, "steps": 10, "warmup": 2, "llm_parsed_share": 0.5,
                                            "answer_format": "span", "traffic": "formats",
                                            "config": {"msgs_per_step_per_gpu": 100}}) + "\n")


def test_gpu_us_per_msg_csv_and_db(tmp_path):
    rows = [("void gemm_fused_kernel<...>(...)", 3, 600_000), ("attn_grouped_kernel(...)", 3, 300_000),
            ("sparse_argmax_kernel(...)", 3, 60_000), ("spec_draft_kernel(...)", 3, 30_000), ("copyBuffer", 1, 10_000)]
    st = tmp_path / "k_kernel_stats.csv"
    with open(st, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs"])
        for r in rows:
            w.writerow(r)
    db = tmp_path / "run_results.db"
    con = sqlite3.connect(db)
    con.execute("CREATE TABLE top_kernels (name TEXT, total_calls INT, total_duration REAL, average REAL, "
                "percentage REAL)")
    con.executemany("INSERT INTO top_kernels VALUES (?, ?, ?, 0, 0)", [(n, c, t / 1e3) for n, c, t in rows])
    con.commit()
    con.close()
    b = tmp_path / "bench.json"
    _bench_line(b)
    outs = []
    for src in (st, db):
        r = subprocess.run([sys.executable, str(ROOT / "scripts/gpu_us_per_msg.py"), str(src), str(b)],
                           capture_output=True, text=True, check=True)
        outs.append(json.loads(r.stdout))
    for o in outs:
        # 1 000 000 ns of kernels over (10 + 2) x 100 x 0.5 = 600 LLM-routed messages
        assert o["llm_msgs"] == 600 and abs(o["gpu_us_per_msg"] - 1000.0 / 600 * 1000 / 1000) < 0.01
        g = o["by_group_us_per_msg"]
        assert g["gemm"] == round(600 / 600, 2) and g["attention"] == 0.5 and g["spec_plan_verify"] == 0.05
    assert outs[0] == outs[1]


def test_cprof_top(tmp_path):
    import cProfile

    d = tmp_path / "cprof"
    d.mkdir()
    for name in ("parser-r0-w0", "parser-r0-w1", "rank0"):
        pr = cProfile.Profile()
        pr.enable()
        sum(i * i for i in range(20000))
        pr.disable()
        pr.dump_stats(str(d / f"{name}.pstats"))
    b = tmp_path / "bench.json"
    _bench_line(b)
    r = subprocess.run([sys.executable, str(ROOT / "scripts/cprof_top.py"), str(d), "--bench", str(b), "--n", "5"],
                       capture_output=True, text=True, check=True)
    assert "## parser processes (2 aggregated)" in r.stdout and "## rank0.pstats" in r.stdout
    assert "us/msg over 1000 msgs" in r.stdout
