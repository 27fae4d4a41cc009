#!/usr/bin/env python3
"""Size a span-pointer answer format before building it (VERDICT r03 next #2a).

Today every copied field is written token by token (the body's own tokens, drafted
by speculative decoding).  A span-pointer format would write each copy field as two
pointer tokens (start / end body position; one "empty" token for a missing field)
and the enum txn_type as now -- no <sep>s, nothing to draft.

Replays gold answers (as if the extractor were exact) on the bench's traffic and
prints, per message: prompt rows, today's answer tokens, today's decode GEMM rows
under continuous batching with the engine's draft policy (scripts/spec_sim.py:
``resume+forced``, water-filled budget of ``--frac`` x rows), today's decode steps;
and the same for the pointer format (one GEMM row and one step per token).

    python scripts/span_sim.py --n 3000 --traffic formats
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--n", type=int, default=3000)
    p.add_argument("--traffic", default="formats")
    p.add_argument("--k", type=int, default=6)
    p.add_argument("--frac", type=float, default=1.25)
    p.add_argument("--batch", type=int, default=4096)
    a = p.parse_args(argv)
    from scripts.spec_sim import clamp, drafts
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.models.train import answer_tokens
    from smsgate_amd.parse.text import normalize_body
    from smsgate_amd.serving.fsm import build_fsm
    from smsgate_amd.utils.synth import generate_traffic

    tok = load_tokenizer()
    fsm = build_fsm(tok, 49152)
    items = [s for s in generate_traffic(a.n, seed=7, traffic=a.traffic) if s.answer]
    exs, prompt = [], 0
    ptr_tokens = 0
    for s in items:
        b = normalize_body(s.body)
        enc = tok.encode_offsets([b])[0]
        ans = answer_tokens(tok, fsm, s.answer, b, enc)
        if ans is None:
            continue
        body = tok.message_ids([b], 128)[0]
        exs.append((body, ans))
        prompt += len(body)
        vals = fsm.split_fields(ans)
        ptr_tokens += len(vals[0]) + sum(2 if v else 1 for v in vals[1:])  # enum as now; [start, end] | [empty]
    strings = tok.token_strings
    delim = [(("," in x) or ("&#" in x) or (";" in x)) and i != tok.sep for i, x in enumerate(strings)]
    delim += [False] * (49152 - len(delim))

    def walk(seq):
        st = fsm.start_state
        for x in seq:
            st = fsm.step_host(st, x)
            if st < 0:
                return -1
        return st

    allowed = lambda seq: walk(seq) >= 0  # noqa: E731
    only = {int(st): int(fsm.allowed[st].nonzero()[0][0]) for st in range(fsm.num_states)
            if fsm.allowed[st].sum() == 1 and st != fsm.done_state}

    def forced(seq):
        st = walk(seq)
        return only.get(st) if st >= 0 else None

    # continuous batching with a shared draft budget (the engine's steady state)
    policy = "resume+forced"
    pool = list(exs)
    live, rows, steps_total, done = [], 0, 0, 0
    budget = math.ceil(a.frac * a.batch)
    msg_steps = []
    while pool or live:
        while pool and len(live) < a.batch:
            body, ans = pool.pop()
            live.append([body, ans, [ans[0]], 1, 1])
        ds = [drafts(policy, r[0], r[2], tok.sep, delim, a.k, allowed, forced) for r in live]
        nds = clamp([len(d) for d in ds], budget, "water")
        rows += len(live) + sum(nds)
        keep = []
        for r, d, nd in zip(live, ds, nds):
            body, ans, out, pos, st = r
            d = d[:nd]
            acc = 0
            while acc < len(d) and pos + acc < len(ans) and d[acc] == ans[pos + acc]:
                acc += 1
            n = min(acc + 1, len(ans) - pos)
            r[2], r[3], r[4] = out + ans[pos:pos + n], pos + n, st + 1
            if r[3] < len(ans):
                keep.append(r)
            else:
                done += 1
                msg_steps.append(r[4])
        live = keep
        steps_total += 1
    m = len(exs)
    ans_tok = sum(len(x[1]) for x in exs) / m
    cur_rows = rows / m
    ptr = ptr_tokens / m
    out = {"traffic": a.traffic, "messages": m, "prompt_rows": round(prompt / m, 1),
           "current": {"answer_tokens": round(ans_tok, 1), "decode_rows": round(cur_rows, 1),
                       "decode_steps": round(sum(msg_steps) / len(msg_steps), 1),
                       "total_rows": round(prompt / m + cur_rows, 1)},
           "span_pointer": {"answer_tokens": round(ptr, 1), "decode_rows": round(ptr, 1), "decode_steps": round(ptr, 1),
                            "total_rows": round(prompt / m + ptr, 1)}}
    out["gemm_rows_change"] = round(out["span_pointer"]["total_rows"] / out["current"]["total_rows"] - 1, 3)
    out["decode_steps_change"] = round(out["span_pointer"]["decode_steps"] / out["current"]["decode_steps"] - 1, 3)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
