"""The native tokenizer (native/csrc/tokfast.cpp) is the library, id for id.

The parser processes encode bodies and decode answers with it (models/fasttok.py);
any divergence would change what the GPU engine sees, so equality is pinned on
every template family, the reference CASES and random Unicode text."""
from __future__ import annotations

import random
import struct

import numpy as np
import pytest

from smsgate_amd.models.fasttok import load_fast_tokenizer, native_available
from smsgate_amd.models.tokenizer import load_tokenizer
from smsgate_amd.parse.text import normalize_body
from smsgate_amd.utils.synth import generate, reference_cases

pytestmark = pytest.mark.skipif(not native_available(), reason="native tokenizer not built")


@pytest.fixture(scope="module")
def toks():
    return load_tokenizer(), load_fast_tokenizer()


def _fuzz(r: random.Random) -> str:
    pools = [
        "abcXYZ", "0123456789", " ", ".,:;-/*$€£₽₾֏'\"()[]", "абвгдЖЩЯ", "\t\n  　 ",
        "٣５१𝟙²½Ⅻ", "&#10;", "<sms><ans><sep>", "é漢字😀́", "'s't're've'm'll'd",
    ]
    out = []
    for _ in range(r.randint(0, 40)):
        p = r.choice(pools)
        out.append(r.choice(p) if r.random() < 0.8 else p)
    if r.random() < 0.2:
        c = r.randint(0x20, 0x2FFFF)
        if not 0xD800 <= c <= 0xDFFF:  # lone surrogates: the library refuses them (see below)
            out.append(chr(c))
    return "".join(out)


def test_equal_to_library_on_every_family(toks):
    tk, ft = toks
    items = generate(4000, seed=71, vocab_name="heldout", families="all") + generate(1000, seed=72)
    bodies = [normalize_body(s.body) for s in items] + reference_cases()
    for b in bodies:
        assert ft.encode(b) == tk.encode(b), b


def test_equal_to_library_on_unicode_fuzz(toks):
    tk, ft = toks
    r = random.Random(1234)
    for _ in range(20000):
        s = _fuzz(r)
        assert ft.encode(s) == tk.encode(s), repr(s)


def test_packed_message_ids_match_message_ids(toks):
    tk, ft = toks
    bodies = [normalize_body(s.body) for s in generate(300, seed=5, vocab_name="heldout", families="all")]
    bodies.append("x " * 300)  # truncated
    want = tk.message_ids(bodies, 128)
    cut, lens, flat = ft.encode_packed(bodies, 128, tk.ans)
    ln = np.frombuffer(lens, dtype=np.uint16)
    ids = np.frombuffer(flat, dtype=np.int32)
    got = np.split(ids, np.cumsum(ln[:-1].astype(np.int64)))
    assert cut == 1 and [g.tolist() for g in got] == want


def test_decode_fields_matches_python(toks):
    tk, ft = toks
    r = random.Random(3)
    seqs = []
    for s in generate(300, seed=8, vocab_name="heldout", families="all"):
        from smsgate_amd.models.train import answer_tokens
        from smsgate_amd.serving.fsm import build_fsm

        fsm = build_fsm(tk, (tk.vocab_size + 63) // 64 * 64) if not seqs else fsm  # noqa: F821
        a = answer_tokens(tk, fsm, s.answer, normalize_body(s.body))
        seqs.append(a)
    seqs += [[], [tk.sep] * 12, [r.randrange(tk.vocab_size) for _ in range(40)], [5, 7, 9]]
    lens = np.array([len(s) for s in seqs], dtype=np.uint16)
    flat = np.array([t for s in seqs for t in s], dtype=np.int32)
    hdr = struct.pack("<cQI", b"R", 1, len(seqs))
    buf = hdr + lens.tobytes() + flat.tobytes()
    assert ft.decode_fields(buf, len(hdr), len(seqs), 9) == tk.decode_fields(seqs, 9)
    with pytest.raises(ValueError):
        ft.decode_fields(buf[:-4], len(hdr), len(seqs), 9)


def test_lone_surrogate_does_not_fail_the_batch(toks):
    tk, ft = toks
    cut, lens, flat = ft.encode_packed(["ok body", "bad \udde2 body", "also ok"], 128, tk.ans)
    ln = np.frombuffer(lens, dtype=np.uint16).tolist()
    ids = np.frombuffer(flat, dtype=np.int32).tolist()
    assert len(ln) == 3 and ids[:ln[0]] == tk.encode("ok body") + [tk.ans]
    assert ids[ln[0] + ln[1]:] == tk.encode("also ok") + [tk.ans]


def test_full_cache_is_emptied_and_refilled_exactly(toks):
    """The pre-token cache empties itself when it reaches its capacity (2^18 entries):
    held-out traffic's one-off names and amounts must not freeze it.  Encodings before,
    across and after the reset equal the library's."""
    tk, ft = toks
    r = random.Random(9)
    # letters only: every word is one pre-token (" WORD"), ~300 k distinct ones
    words = ["".join(r.choice("ABCDEFGHKLMNPRSTUVZ") for _ in range(r.randint(5, 9))) for _ in range(300000)]
    probe = "Покупка 1 500,00 RUB в SHOP CITY, ул. LENINA 5; баланс 12 345,67 RUB"
    want = tk.encode(probe)
    assert ft.encode(probe) == want
    for i in range(0, len(words), 5000):
        ft.encode(" ".join(words[i:i + 5000]))
    # more distinct pre-tokens than the capacity went in: a cache that stopped inserting
    # when full would sit at exactly 2^18 entries
    assert 0 < ft.cache_size() < 2 ** 18
    assert ft.encode(probe) == want
    sample = " ".join(words[-50:])
    assert ft.encode(sample) == tk.encode(sample)
