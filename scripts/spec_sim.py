#!/usr/bin/env python3
"""CPU simulation of the speculative-decode draft policy (csrc/spec_kernels.hip).

Replays gold answers as if the extractor decoded them exactly: each step emits
the accepted prefix of the row's drafts plus one model token.  Prints decode
steps per message and tokens per row-step for each draft policy, so a policy
change can be judged before it is written as a kernel.

    python scripts/spec_sim.py --n 2000 --k 4
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def find_anchor(body, t, prev):
    if prev is not None:
        for q in range(1, len(body)):
            if body[q] == t and body[q - 1] == prev:
                return q
    for q in range(len(body)):
        if body[q] == t:
            return q
    return -1


def drafts(policy, body, out, sep, delim, K, allowed, forced=None):
    """Draft tokens after emitted prefix ``out`` (``allowed(out + d)``: schema check;
    ``forced(seq)``: the only token the schema allows after ``seq``, else None)."""
    t = out[-1] if out else None
    if t is None:
        return []
    if forced is not None and "forced" in policy:
        d = []
        while len(d) < K and (f := forced(out + d)) is not None:
            d.append(f)
        if d:
            rest = drafts(policy.replace("forced", ""), body, out + d, sep, delim, K - len(d), allowed, forced)
            return d + rest if len(d) < K else d
    if t == sep:
        if "scan" in policy:
            d = drafts(policy.replace("scan", ""), body, out, sep, delim, K, allowed, forced)
            if d:
                return d
            for q in range(len(body)):
                x = body[q]
                if not delim[x] and allowed(out + [x]):
                    return [x] + drafts(policy.replace("scan", ""), body, out + [x], sep, delim, K - 1, allowed, forced)[:K - 1]
            return []
        if "resume" not in policy or len(out) < 2:
            return []
        # field start: resume the body right after the previous field's last copied token
        prev_tok = out[-2]
        if prev_tok == sep:
            return []
        prev2 = out[-3] if len(out) >= 3 and out[-3] != sep else None
        j = find_anchor(body, prev_tok, prev2)
        if j < 0:
            return []
        q0 = j + 1
        while q0 < len(body) and delim[body[q0]]:
            q0 += 1
        j = q0 - 1
    else:
        prev = out[-2] if len(out) >= 2 and out[-2] != sep else None
        j = find_anchor(body, t, prev)
        if j < 0:
            return []
    d = []
    q = j + 1
    while len(d) < K and q < len(body):
        x = sep if delim[body[q]] else body[q]
        if not allowed(out + d + [x]):
            if ("implicit" in policy or "resume" in policy) and x != sep and allowed(out + d + [sep]):
                d.append(sep)
                if len(d) < K and allowed(out + d + [x]):
                    d.append(x)
                    q += 1
                    continue
            break
        d.append(x)
        q += 1
        if x == sep and "base" in policy:
            break
    return d


def clamp(nds, budget, fill):
    if fill == "order":
        out, left = [], budget
        for n in nds:
            out.append(min(n, left))
            left -= out[-1]
        return out
    c = 0
    for cc in range(1, max(nds, default=0) + 1):
        if sum(min(n, cc) for n in nds) <= budget:
            c = cc
    extra = budget - sum(min(n, c) for n in nds)
    out = []
    for n in nds:
        f = min(n, c)
        if n > c and extra > 0:
            f += 1
            extra -= 1
        out.append(f)
    return out


def batch_sim(a, policy, exs, sep, delim, allowed, forced):
    """Continuous batching: ``a.batch`` live rows, finished rows replaced at once."""
    import math

    pool = list(exs)
    live = []  # [body, ans, out, pos]
    steps = done = 0
    budget = math.ceil(a.frac * a.batch)
    while pool or live:
        while pool and len(live) < a.batch:
            body, ans = pool.pop()
            live.append([body, ans, [ans[0]], 1])
        ds = [drafts(policy, r[0], r[2], sep, delim, a.k, allowed, forced) for r in live]
        if a.fill == "tiered":
            # tier A: the round-2 first-cut draft (forced tokens + copy to the first <sep>)
            nas = []
            for r, d in zip(live, ds):
                da = drafts("base+forced", r[0], r[2], sep, delim, a.k, allowed, forced)
                n = 0
                while n < min(len(da), len(d)) and da[n] == d[n]:
                    n += 1
                nas.append(n)
            fa = clamp(nas, budget, "water")
            left = budget - sum(fa)
            ext = [len(d) - na if f == na else 0 for d, na, f in zip(ds, nas, fa)]
            fb = clamp(ext, left, "water")
            nds = [x + y for x, y in zip(fa, fb)]
        else:
            nds = clamp([len(d) for d in ds], budget, a.fill)
        keep = []
        for r, d, n_d in zip(live, ds, nds):
            body, ans, out, pos = r
            d = d[:n_d]
            acc = 0
            while acc < len(d) and pos + acc < len(ans) and d[acc] == ans[pos + acc]:
                acc += 1
            n = min(acc + 1, len(ans) - pos)
            r[2] = out + ans[pos:pos + n]
            r[3] = pos + n
            if r[3] < len(ans):
                keep.append(r)
            else:
                done += 1
        live = keep
        steps += 1
        if len(pool) == 0 and len(live) < a.batch // 4:
            break  # drain tail: not steady state
    rate = done / steps
    print(f"{policy:18s} K={a.k} frac={a.frac} fill={a.fill}: msgs/step {rate:7.2f}  "
          f"per pseudo-row {rate / (a.batch + budget):.4f}")


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--n", type=int, default=2000)
    p.add_argument("--k", type=int, default=4)
    p.add_argument("--seed", type=int, default=11)
    p.add_argument("--vocab", default="heldout")
    p.add_argument("--policies", default="base,continue,implicit,resume,resume+forced,resume+forced+scan")
    p.add_argument("--batch", type=int, default=0,
                   help="> 0: continuous batch of this many rows sharing a draft budget of --frac x rows per step")
    p.add_argument("--frac", type=float, default=1.25)
    p.add_argument("--fill", default="water", choices=["water", "order", "tiered"], help="budget clamp (spec_scan_kernel)")
    a = p.parse_args(argv)
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.models.train import make_examples
    from smsgate_amd.serving.fsm import build_fsm

    tok = load_tokenizer()
    fsm = build_fsm(tok, 49152)
    exs = make_examples(tok, fsm, a.n, a.seed, vocab_name=a.vocab)
    strings = tok.token_strings
    delim = [(("," in s) or ("&#" in s) or (";" in s)) and i != tok.sep for i, s in enumerate(strings)]
    delim += [False] * (49152 - len(delim))

    def walk(seq):
        s = fsm.start_state
        for x in seq:
            s = fsm.step_host(s, x)
            if s < 0:
                return -1
        return s

    def allowed(seq):
        return walk(seq) >= 0

    only = {int(st): int(fsm.allowed[st].nonzero()[0][0]) for st in range(fsm.num_states)
            if fsm.allowed[st].sum() == 1}

    def forced(seq):
        st = walk(seq)
        return None if st < 0 or st == fsm.done_state else only.get(st)

    if a.batch:
        for policy in a.policies.split(","):
            batch_sim(a, policy, exs, tok.sep, delim, allowed, forced)
        return 0
    for policy in a.policies.split(","):
        steps = toks = 0
        for body, ans in exs:
            out = [ans[0]]  # the prefill emits the first token
            pos = 1
            while pos < len(ans):
                d = drafts(policy, body, out, tok.sep, delim, a.k, allowed, forced)
                acc = 0
                while acc < len(d) and pos + acc < len(ans) and d[acc] == ans[pos + acc]:
                    acc += 1
                n = min(acc + 1, len(ans) - pos)
                out += ans[pos:pos + n]
                pos += n
                steps += 1
                toks += n
        print(f"{policy:9s} steps/msg {steps / len(exs):6.2f}  tokens/row-step {toks / steps:5.2f}  "
              f"(answers {sum(len(x[1]) for x in exs) / len(exs):.1f} tokens)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
