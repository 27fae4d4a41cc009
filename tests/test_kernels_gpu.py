"""Numerics of the HIP kernels vs plain PyTorch fp32 references (MI355X only)."""
import math

import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]

from smsgate_amd import ops  # noqa: E402

DEV = "cuda"


def _bf(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


def test_library_loads_from_tree():
    lib = ops.load_library()
    assert lib.sg_version() == 1
    assert "smsgate_amd/ops/_lib" in lib._name


@pytest.mark.parametrize("T,H", [(1, 576), (7, 576), (300, 576), (33, 1024)])
def test_rmsnorm_residual(T, H):
    res = _bf(T, H, seed=1)
    x = _bf(T, H, seed=2)
    w = _bf(H, seed=3) + 1
    res0 = res.clone()
    out = ops.rmsnorm_residual(res, w, 1e-5, x=x)
    new_res = (res0.float() + x.float()).to(torch.bfloat16)
    assert torch.equal(res, new_res)
    ref = ops.ref_rmsnorm(new_res, w, 1e-5)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    out2 = ops.rmsnorm_residual(res0.clone(), w, 1e-5)
    torch.testing.assert_close(out2.float(), ops.ref_rmsnorm(res0, w, 1e-5), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("T,I", [(1, 1536), (129, 1536), (5, 64)])
def test_silu_mul(T, I):
    gu = _bf(T, 2 * I, scale=3.0)
    out = ops.silu_mul(gu)
    torch.testing.assert_close(out.float(), ops.ref_silu_mul(gu), atol=3e-2, rtol=2e-2)


def test_rope_qkv_cache():
    T, nh, nkv, D, S, Lmax, p0 = 37, 9, 3, 64, 5, 64, 11
    qkv = _bf(T, (nh + 2 * nkv) * D)
    pos = torch.randint(0, Lmax, (T,), dtype=torch.int32, device=DEV)
    slot = torch.randint(0, S, (T,), dtype=torch.int32, device=DEV)
    # unique (slot, pos) pairs so writes don't collide
    pairs = torch.randperm(S * Lmax)[:T]
    slot = (pairs // Lmax).to(torch.int32).to(DEV)
    pos = (pairs % Lmax).to(torch.int32).to(DEV)
    cs = ops.rope_table(p0 + Lmax + 1, D, 1e5, DEV)
    q = torch.empty(T, nh, D, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(S, nkv, Lmax, D, dtype=torch.bfloat16, device=DEV)
    vt = torch.zeros(*ops.vt_shape(S, nkv, D, Lmax), dtype=torch.bfloat16, device=DEV)
    ops.rope_qkv_cache(qkv, pos, slot, cs, q, kc, vt, nh, nkv, D, p0)
    qf, kf, vf = qkv.float().split([nh * D, nkv * D, nkv * D], -1)
    absp = (pos + p0).long()
    qr = ops.ref_rope(qf.view(T, nh, D), absp, 1e5)
    kr = ops.ref_rope(kf.view(T, nkv, D), absp, 1e5)
    torch.testing.assert_close(q.float(), qr, atol=2e-2, rtol=2e-2)
    sl, ps = slot.long(), pos.long()
    torch.testing.assert_close(kc[sl, :, ps, :].float(), kr, atol=2e-2, rtol=2e-2)
    got_v = ops.vt_to_rows(vt)[sl, :, ps, :]  # [T, nkv, D]
    assert torch.equal(got_v.float(), vf.view(T, nkv, D))


def _ref_seq_attention(qb, own_k, own_v, pk, pv, P0, q_off, scale):
    """qb [nq, nh, D]; own_k/v [nown, nkv, D]; pk/pv [P0, nkv, D]; q_off[i] = own offset of query i."""
    nq, nh, D = qb.shape
    nkv = own_k.shape[1]
    G = nh // nkv
    out = torch.empty(nq, nh, D, device=qb.device)
    nown = own_k.shape[0]
    keys_k = torch.cat([pk, own_k], 0)
    keys_v = torch.cat([pv, own_v], 0)
    kidx = torch.arange(P0 + nown, device=qb.device)
    mask = (kidx[None, :] < P0) | ((kidx[None, :] - P0) <= torch.as_tensor(q_off, device=qb.device)[:, None])
    for h in range(nh):
        kh = h // G
        out[:, h] = ops.ref_attention(qb[:, h], keys_k[:, kh], keys_v[:, kh], mask, scale)
    return out


@pytest.mark.parametrize("impl", ["gqa", "gqa_ks2", "per_head", "multi", "st", "st32", "st64", "st32pf", "stpf", "st64pf"])
@pytest.mark.parametrize("heads", [(9, 3), (4, 2), (4, 4), (8, 2)])
@pytest.mark.parametrize("P0", [0, 20, 75])  # 0 / 20: merged prefix + own key stream; 75: prefix tiles first
def test_attn_prefill(P0, heads, impl):
    nh, nkv = heads
    D, S, Lmax = 64, 6, 200
    ops.set_prefill_impl("gqa" if impl.startswith("gqa") else impl)
    ops.set_prefill_split(2 if impl == "gqa_ks2" else 1)
    P0pad = (P0 + 31) // 32 * 32
    lens = [1, 17, 40, 63, 5]
    starts = [0, 0, 3, 0, 30]  # own offset of each chunk's first query (chunked prefill)
    rows = [4, 0, 2, 5, 1]
    T = sum(lens)
    q = _bf(T, nh, D, seed=4)
    kc = _bf(S, nkv, Lmax, D, seed=5)
    vrows = _bf(S, nkv, Lmax, D, seed=6)
    vt = ops.rows_to_vt(vrows)
    pk = torch.zeros(nkv, P0pad, D, dtype=torch.bfloat16, device=DEV)
    pvrows = torch.zeros(nkv, P0pad, D, dtype=torch.bfloat16, device=DEV)
    if P0:
        pk[:, :P0] = _bf(nkv, P0, D, seed=7)
        pvrows[:, :P0] = _bf(nkv, P0, D, seed=8)
    pvt = ops.rows_to_vt(pvrows)
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(lens), 0)), dtype=torch.int32, device=DEV)
    qs = torch.tensor(starts, dtype=torch.int32, device=DEV)
    sl = torch.tensor(rows, dtype=torch.int32, device=DEV)
    out = torch.empty(T, nh * D, dtype=torch.bfloat16, device=DEV)
    scale = 1 / math.sqrt(D)
    try:
        ops.attn_prefill(q, cu, qs, sl, max(lens), kc, vt, pk, pvt, P0, out, scale)
    finally:
        ops.set_prefill_impl("auto")
        ops.set_prefill_split(1)
    o = 0
    for n, st, r in zip(lens, starts, rows):
        nown = st + n
        own_k = kc[r, :, :nown].permute(1, 0, 2).float()
        own_v = vrows[r, :, :nown].permute(1, 0, 2).float()
        ref = _ref_seq_attention(q[o:o + n].float(), own_k, own_v, pk[:, :P0].permute(1, 0, 2).float(),
                                 pvrows[:, :P0].permute(1, 0, 2).float(), P0, list(range(st, st + n)), scale)
        torch.testing.assert_close(out[o:o + n].float().view(n, nh, D), ref, atol=3e-2, rtol=3e-2)
        o += n


def test_attn_prefill_auto_width_is_bitwise_stable():
    """auto switches the transposed kernel from 32 to 64 columns per wave at 1 024
    sequences (the qa engine's batches).  A column's arithmetic does not depend on the
    width, so outputs are bit for bit the same.  A message's answer then cannot depend
    on the batch it was packed into."""
    nh, nkv, D, Lmax, P0 = 9, 3, 64, 192, 4
    g = torch.Generator(device="cpu").manual_seed(3)
    lens = torch.randint(45, 56, (1100,), generator=g).tolist()
    S, T = len(lens), sum(lens)
    q = _bf(T, nh, D, seed=31)
    kc = _bf(S, nkv, Lmax, D, seed=32)
    vt = ops.rows_to_vt(_bf(S, nkv, Lmax, D, seed=33))
    pk = torch.zeros(nkv, 32, D, dtype=torch.bfloat16, device=DEV)
    pk[:, :P0] = _bf(nkv, P0, D, seed=34)
    pvt = ops.rows_to_vt(pk.clone())
    cu = torch.tensor([0] + torch.cumsum(torch.tensor(lens), 0).tolist(), dtype=torch.int32, device=DEV)
    qs = torch.zeros(S, dtype=torch.int32, device=DEV)
    sl = torch.arange(S, dtype=torch.int32, device=DEV)
    outs = {}
    try:
        for impl in ("st32", "st64", "auto"):
            ops.set_prefill_impl(impl)
            out = torch.empty(T, nh * D, dtype=torch.bfloat16, device=DEV)
            ops.attn_prefill(q, cu, qs, sl, max(lens), kc, vt, pk, pvt, P0, out, 1 / math.sqrt(D))
            outs[impl] = out
    finally:
        ops.set_prefill_impl("auto")
    assert torch.equal(outs["st32"], outs["st64"]) and torch.equal(outs["auto"], outs["st64"])


@pytest.mark.parametrize("impl", ["grouped", "grouped_h", "grouped6", "grouped_pf", "cascade", "mfma", "mfma_v1", "valu", "split2", "split4",
                                  "split8"])
@pytest.mark.parametrize("P0", [0, 20, 75])
def test_attn_decode(P0, impl):
    nh, nkv, D, S, Lmax = 9, 3, 64, 8, 224  # MFMA decode tiles need Lmax % 32 == 0
    P0pad = (P0 + 31) // 32 * 32
    B = 6
    q = _bf(B, nh, D, seed=9)
    kc = _bf(S, nkv, Lmax, D, seed=10)
    vrows = _bf(S, nkv, Lmax, D, seed=11)
    vt = ops.rows_to_vt(vrows)
    pk = torch.zeros(nkv, P0pad, D, dtype=torch.bfloat16, device=DEV)
    pvrows = torch.zeros(nkv, P0pad, D, dtype=torch.bfloat16, device=DEV)
    if P0:
        pk[:, :P0] = _bf(nkv, P0, D, seed=12)
        pvrows[:, :P0] = _bf(nkv, P0, D, seed=13)
    pvt = ops.rows_to_vt(pvrows)
    pos = torch.tensor([0, 1, 7, 8, 100, 223], dtype=torch.int32, device=DEV)  # 223: own == Lmax
    slot = torch.tensor([3, 0, 7, 1, 2, 5], dtype=torch.int32, device=DEV)
    out = torch.full((B, nh * D), 7.0, dtype=torch.bfloat16, device=DEV)
    scale = 1 / math.sqrt(D)
    done = torch.zeros(B, dtype=torch.int32, device=DEV)
    done[2] = 1  # finished rows are skipped
    ops.attn_decode(q, pos, slot, kc, vt, pk, pvt, P0, out, scale, done=done, impl=impl)
    for b in range(B):
        if b == 2:
            assert torch.all(out[b] == 7.0)
            continue
        p, r = int(pos[b]), int(slot[b])
        own_k = kc[r, :, : p + 1].permute(1, 0, 2).float()
        own_v = vrows[r, :, : p + 1].permute(1, 0, 2).float()
        ref = _ref_seq_attention(q[b:b + 1].float(), own_k, own_v, pk[:, :P0].permute(1, 0, 2).float(),
                                 pvrows[:, :P0].permute(1, 0, 2).float(), P0, [p], scale)
        torch.testing.assert_close(out[b].float().view(1, nh, D), ref, atol=2e-2, rtol=2e-2)


def test_fsm_sample_greedy_and_transitions():
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.serving.fsm import build_fsm

    tk = load_tokenizer()
    V = 49152
    fsm = build_fsm(tk, V).to_device(DEV)
    B = 64
    logits = _bf(B, V, scale=3.0, seed=14)
    states_h = torch.randint(0, fsm.num_states - 1, (B,))
    state = states_h.to(torch.int32).to(DEV)
    tok = torch.zeros(B, dtype=torch.int32, device=DEV)
    out_buf = torch.zeros(B, 8, dtype=torch.int32, device=DEV)
    out_len = torch.zeros(B, dtype=torch.int32, device=DEV)
    done = torch.zeros(B, dtype=torch.int32, device=DEV)
    done[0] = 1
    pos = torch.zeros(B, dtype=torch.int32, device=DEV)
    slot = torch.arange(B, dtype=torch.int32, device=DEV)
    ops.fsm_sample(logits, fsm, state, tok, out_buf, out_len, done, pos, slot, 0.0, 0)
    allowed = torch.from_numpy(fsm.allowed)
    lf = logits.float().cpu()
    for b in range(1, B):
        s = int(states_h[b])
        masked = lf[b].masked_fill(~allowed[s], float("-inf"))
        exp_tok = int(masked.argmax())
        assert int(tok[b]) == exp_tok and int(out_buf[b, 0]) == exp_tok and int(out_len[b]) == 1
        ns = fsm.step_host(s, exp_tok)
        assert int(state[b]) == (ns if ns >= 0 else fsm.done_state)
    assert int(out_len[0]) == 0  # done rows untouched
    # temperature sampling stays inside the mask
    state2 = states_h.to(torch.int32).to(DEV)
    done.zero_()
    ops.fsm_sample(logits, fsm, state2, tok, out_buf, out_len.zero_(), done, pos, slot, 1.0, 123)
    for b in range(B):
        assert allowed[int(states_h[b]), int(tok[b])]


def _tile_cases(shapes):
    """(cfg, *shape) for every tile config whose BN divides N (others cannot run it)."""
    return [(cfg, *s) for cfg in sorted(ops.GEMM_TILES) for s in shapes
            if cfg not in ops.GEMM_SWIGLU_ONLY | ops.GEMM_RESID_ONLY and s[1] % ops.GEMM_TILES[cfg][1] == 0]


@pytest.mark.parametrize("cfg,M,N,K", _tile_cases([(1, 128, 64), (100, 576, 576), (777, 960, 576),
                                                   (256, 3072, 576), (130, 576, 1536), (64, 8192, 576)]))
def test_gemm_store_and_norm(cfg, M, N, K):
    a = _bf(M, K, seed=11)
    w = _bf(N, K, scale=K ** -0.5, seed=12)
    nw = _bf(K, scale=0.1, seed=13) + 1
    out = ops.gemm(a, w, cfg=cfg)
    torch.testing.assert_close(out.float(), ops.ref_gemm(a, w), atol=3e-2, rtol=2e-2)
    out_n = ops.gemm(a, ops.fold_norm(w, nw), norm_eps=1e-5, cfg=cfg)
    torch.testing.assert_close(out_n.float(), ops.ref_gemm(a, w, norm_eps=1e-5, norm_w=nw), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("cfg,M,N,K", _tile_cases([(1, 576, 1536), (333, 576, 1536), (2048, 576, 1536)])
                         + [(c, M, 576, K) for c in sorted(ops.GEMM_RESID_ONLY)
                            for M, K in ((1, 1536), (333, 1536), (2048, 576), (70000, 1536))])
def test_gemm_residual_inplace(cfg, M, N, K):
    a = _bf(M, K, seed=21)
    w = _bf(N, K, scale=K ** -0.5, seed=22)
    x = _bf(M, N, seed=23)
    ref = (x.float() + (a.float() @ w.float().t()).to(torch.bfloat16).float())
    ops.gemm(a, w, epi="resid", resid=x, cfg=cfg)  # in place
    torch.testing.assert_close(x.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("cfg", sorted(set(ops.GEMM_TILES) - ops.GEMM_NO_SWIGLU))
@pytest.mark.parametrize("M", [5, 640])
def test_gemm_swiglu_norm(cfg, M):
    K, I = 576, 1536
    bm, bn = ops.GEMM_TILES[cfg]
    a = _bf(M, K, seed=31)
    gu = _bf(2 * I, K, scale=K ** -0.5, seed=32)
    nw = _bf(K, scale=0.1, seed=33) + 1
    w = ops.interleave_gate_up(ops.fold_norm(gu, nw))
    out = ops.gemm(a, w, epi="swiglu", norm_eps=1e-5, cfg=cfg)
    assert out.shape == (M, I)
    ref = ops.ref_gemm(a, gu, epi="swiglu", norm_eps=1e-5, norm_w=nw)
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)


def test_gemm_strided_a_and_bad_shapes():
    a_full = _bf(50, 640, seed=41)
    a = a_full[:, :576]  # row stride 640 > K
    w = _bf(128, 576, seed=42)
    torch.testing.assert_close(ops.gemm(a, w).float(), ops.ref_gemm(a, w), atol=5e-2, rtol=2e-2)
    with pytest.raises(ValueError):
        ops.gemm(_bf(4, 100), _bf(64, 100))


@pytest.mark.parametrize("cfg", [1, 3, 5, 17, 18, 23, 26, 28])
@pytest.mark.parametrize("M", [1, 77, 1000, 9216])
def test_gemm_qkv_rope_matches_unfused(cfg, M):
    nh, nkv, D, S, Lmax, K, p0 = 9, 3, 64, max(1024, M), 192, 576, 75
    x = _bf(M, K, seed=51)
    w = _bf((nh + 2 * nkv) * D, K, scale=K ** -0.5, seed=52)
    g = torch.Generator(device="cpu").manual_seed(53)
    pos = torch.randint(0, Lmax, (M,), generator=g, dtype=torch.int32).to(DEV)
    slot = torch.randperm(S, generator=g)[:M].to(torch.int32).to(DEV)
    cs = ops.rope_table(p0 + Lmax + 1, D, 100000.0, DEV)
    caches = []
    for fused in (True, False):
        kc = torch.zeros(S, nkv, Lmax, D, dtype=torch.bfloat16, device=DEV)
        vt = torch.zeros(*ops.vt_shape(S, nkv, D, Lmax), dtype=torch.bfloat16, device=DEV)
        q = torch.zeros(M, nh, D, dtype=torch.bfloat16, device=DEV)
        if fused:
            ops.gemm_qkv_rope(x, w, 1e-5, pos, slot, cs, q, kc, vt, nh, nkv, p0, cfg=cfg)
        else:
            qkv = ops.gemm(x, w, norm_eps=1e-5, cfg=cfg)
            ops.rope_qkv_cache(qkv, pos, slot, cs, q, kc, vt, nh, nkv, D, p0)
        caches.append((q, kc, vt))
    for a, b in zip(*caches):
        torch.testing.assert_close(a.float(), b.float(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("cfg", [1, 3, 17, 23, 28])
def test_gemm_qkv_rope_packed_sequences(cfg):
    """Packed prefill rows (sequences of 1..70 tokens at positions 0.., one slot each):
    the epilogue writes whole 8-position V^T blocks as 16-B chunks when a tile holds all
    8 rows of one, element by element at sequence and tile edges -- the caches equal the
    unfused path's exactly."""
    nh, nkv, D, S, Lmax, K, p0 = 9, 3, 64, 512, 192, 576, 6
    g = torch.Generator(device="cpu").manual_seed(61)
    lens = torch.randint(1, 71, (300,), generator=g)
    M = int(lens.sum())
    pos = torch.cat([torch.arange(int(n)) for n in lens]).to(torch.int32).to(DEV)
    slot = torch.repeat_interleave(torch.randperm(S, generator=g)[:300], lens).to(torch.int32).to(DEV)
    x = _bf(M, K, seed=62)
    w = _bf((nh + 2 * nkv) * D, K, scale=K ** -0.5, seed=63)
    cs = ops.rope_table(p0 + Lmax + 1, D, 100000.0, DEV)
    caches = []
    for fused in (True, False):
        kc = torch.zeros(S, nkv, Lmax, D, dtype=torch.bfloat16, device=DEV)
        vt = torch.zeros(*ops.vt_shape(S, nkv, D, Lmax), dtype=torch.bfloat16, device=DEV)
        q = torch.zeros(M, nh, D, dtype=torch.bfloat16, device=DEV)
        if fused:
            ops.gemm_qkv_rope(x, w, 1e-5, pos, slot, cs, q, kc, vt, nh, nkv, p0, cfg=cfg)
        else:
            qkv = ops.gemm(x, w, norm_eps=1e-5, cfg=cfg)
            ops.rope_qkv_cache(qkv, pos, slot, cs, q, kc, vt, nh, nkv, D, p0)
        caches.append((q, kc, vt))
    (qa, ka, va), (qb, kb, vb) = caches
    assert torch.equal(va, vb)  # V^T: copied values, exact
    torch.testing.assert_close(qa.float(), qb.float(), atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(ka.float(), kb.float(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("cfg", [0, 3, 17])
@pytest.mark.parametrize("M", [1, 77, 700])
def test_gemm_argmax_matches_logits_path(cfg, M):
    """lm_head GEMM with the fused FSM-masked arg-max (EPI 4) == the logits path:
    same-kernel bf16 logits (ops.gemm with the norm prologue) + fsm_sample's greedy
    pick; fsm_commit then makes the same FSM step as fsm_sample."""
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.serving.fsm import build_fsm

    tk = load_tokenizer()
    V, K = (tk.vocab_size + 127) // 128 * 128, 576
    fsm = build_fsm(tk, V).to_device(DEV)
    a = _bf(M, K, seed=31)
    w = _bf(V, K, scale=0.05, seed=32)
    states_h = torch.randint(0, fsm.num_states, (M,))
    row_state = states_h.to(torch.int32).to(DEV)
    best = torch.zeros(M + 3, dtype=torch.int64, device=DEV)
    ops.gemm_argmax(a, w, row_state, fsm, best, norm_eps=1e-5, cfg=cfg)
    logits = ops.gemm(a, w, norm_eps=1e-5)
    args = [torch.zeros(M, dtype=torch.int32, device=DEV) for _ in range(5)]  # tok, out_len, done, pos, slot
    out_a = torch.zeros(M, 4, dtype=torch.int32, device=DEV)
    st_a = row_state.clone()
    ops.fsm_sample(logits, fsm, st_a, args[0], out_a, args[1], args[2], args[3], args[4], 0.0, 0)
    tok_b = torch.zeros(M, dtype=torch.int32, device=DEV)
    out_b = torch.zeros(M, 4, dtype=torch.int32, device=DEV)
    len_b = torch.zeros(M, dtype=torch.int32, device=DEV)
    st_b = row_state.clone()
    ops.fsm_commit(best, fsm, st_b, tok_b, out_b, len_b, torch.zeros(M, dtype=torch.int32, device=DEV),
                   torch.zeros(M, dtype=torch.int32, device=DEV), M)
    assert torch.equal(args[0], tok_b) and torch.equal(out_a, out_b) and torch.equal(st_a, st_b)
    assert torch.equal(args[1], len_b)
    # and against a plain fp32 masked arg-max of the same bf16 logits
    allowed = torch.from_numpy(fsm.allowed)
    lf = logits.float().cpu()
    for b in range(0, M, max(1, M // 13)):
        s = int(states_h[b])
        if allowed[s].any():
            assert int(tok_b[b]) == int(lf[b].masked_fill(~allowed[s], float("-inf")).argmax())


@pytest.mark.parametrize("cfg", [1, 3, 17, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36])
@pytest.mark.parametrize("M", [5, 333, 2048])
def test_gemm_producer_norm(cfg, M):
    """Residual GEMM with ``ss_out`` writes per-N-tile x² partials of the rows it
    stores; norm GEMMs given them (``ss_in``: SwiGLU, QKV+RoPE, lm_head arg-max)
    match the same GEMMs accumulating x² themselves, and the fp32 reference."""
    H, I, nh, nkv, D, S, Lmax, p0 = 576, 1536, 9, 3, 64, 4096, 192, 20
    a = _bf(M, H, seed=61)
    wo = _bf(H, H, scale=H ** -0.5, seed=62)
    x = _bf(M, H, seed=63)
    ss = ops.ss_buffer(M + 7, DEV)
    x0 = x.clone()
    ops.gemm(a, wo, epi="resid", resid=x, cfg=cfg, ss_out=ss)
    bn = ops.GEMM_TILES[cfg][1]
    parts = H // (96 if bn % 96 == 0 else bn)  # 96- and 192-wide tiles both write 96-column parts
    assert torch.count_nonzero(ss[parts:]) == 0 and torch.count_nonzero(ss[:, M:]) == 0
    if bn % 96 == 0 and cfg != 21:  # ... and the same partials, bit for bit, as the 128x96 tile
        x21, ss21 = x0.clone(), ops.ss_buffer(M + 7, DEV)
        ops.gemm(a, wo, epi="resid", resid=x21, cfg=21, ss_out=ss21)
        assert torch.equal(x21, x) and torch.equal(ss21, ss)
    torch.testing.assert_close(ss[:, :M].sum(0), x.float().pow(2).sum(1), rtol=1e-4, atol=1e-3)
    nw = _bf(H, scale=0.1, seed=64) + 1
    gu = ops.interleave_gate_up(ops.fold_norm(_bf(2 * I, H, scale=H ** -0.5, seed=65), nw))
    own = ops.gemm(x, gu, epi="swiglu", norm_eps=1e-5)
    ext = ops.gemm(x, gu, epi="swiglu", norm_eps=1e-5, ss_in=ss)
    torch.testing.assert_close(ext.float(), own.float(), atol=1e-2, rtol=1e-2)
    # QKV + RoPE + KV write
    wq = _bf((nh + 2 * nkv) * D, H, scale=H ** -0.5, seed=66)
    g = torch.Generator(device="cpu").manual_seed(67)
    pos = torch.randint(0, Lmax, (M,), generator=g, dtype=torch.int32).to(DEV)
    slot = torch.randperm(S, generator=g)[:M].to(torch.int32).to(DEV)
    cs = ops.rope_table(p0 + Lmax + 1, D, 100000.0, DEV)
    outs = []
    for ss_in in (None, ss):
        kc = torch.zeros(S, nkv, Lmax, D, dtype=torch.bfloat16, device=DEV)
        vt = torch.zeros(*ops.vt_shape(S, nkv, D, Lmax), dtype=torch.bfloat16, device=DEV)
        q = torch.zeros(M, nh, D, dtype=torch.bfloat16, device=DEV)
        ops.gemm_qkv_rope(x, wq, 1e-5, pos, slot, cs, q, kc, vt, nh, nkv, p0, ss_in=ss_in)
        outs.append((q, kc, vt))
    for u, v in zip(*outs):
        torch.testing.assert_close(u.float(), v.float(), atol=1e-2, rtol=1e-2)
    # lm_head arg-max: the keys' values agree to bf16 rounding of the logits
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.serving.fsm import build_fsm

    tk = load_tokenizer()
    V = (tk.vocab_size + 127) // 128 * 128
    fsm = build_fsm(tk, V).to_device(DEV)
    w = _bf(V, H, scale=0.05, seed=68)
    row_state = torch.full((M,), fsm.start_state, dtype=torch.int32, device=DEV)
    keys = []
    for ss_in in (None, ss):
        best = torch.zeros(M, dtype=torch.int64, device=DEV)
        ops.gemm_argmax(x, w, row_state, fsm, best, norm_eps=1e-5, ss_in=ss_in)
        keys.append(best)
    same = (keys[0] == keys[1]).float().mean().item()
    assert same >= 0.95, same  # a different fp32 sum order may flip a near-tie's bf16 rounding
    with pytest.raises(ValueError):
        ops.gemm(a, wo, epi="store", ss_out=ss)


@pytest.mark.parametrize("P0,max_q,merge", [(0, 5, 1), (20, 5, 1), (20, 9, 1), (20, 9, 0), (75, 5, 1), (75, 9, 1)])
def test_attn_spec_matches_grouped_bitwise(P0, max_q, merge):
    """attn_spec (one wave per row, all its drafts) == the grouped decode kernel on
    the same pseudo-rows, bit for bit, and == an fp32 reference; finished rows
    (row_nd = -1) untouched.  max_q = 9: 27 columns, two MFMA column blocks per wave.
    P0 % 4 == 0 walks the prefix and own keys as one tile stream (ops.set_attn_merge),
    including the clamped last tile of a full slot in the last slot (215 + 8 drafts)."""
    ops.set_attn_merge(bool(merge))
    try:
        _spec_vs_grouped(P0, max_q)
    finally:
        ops.set_attn_merge(True)


def _spec_vs_grouped(P0, max_q):
    nh, nkv, D, S, Lmax = 9, 3, 64, 8, 224
    P0pad = (P0 + 31) // 32 * 32
    kc = _bf(S, nkv, Lmax, D, seed=20)
    vrows = _bf(S, nkv, Lmax, D, seed=21)
    vt = ops.rows_to_vt(vrows)
    pk = torch.zeros(nkv, P0pad, D, dtype=torch.bfloat16, device=DEV)
    pvrows = torch.zeros(nkv, P0pad, D, dtype=torch.bfloat16, device=DEV)
    if P0:
        pk[:, :P0] = _bf(nkv, P0, D, seed=22)
        pvrows[:, :P0] = _bf(nkv, P0, D, seed=23)
    pvt = ops.rows_to_vt(pvrows)
    # rows: (pos, slot, drafts, done); pos + drafts < Lmax
    rows = [(0, 3, 4, 0), (14, 0, 2, 0), (30, 7, 4, 1), (31, 1, 0, 0), (100, 2, 3, 0), (219, 5, 4, 0), (47, 6, 1, 0)]
    if max_q > 5:
        rows += [(60, 4, 8, 0), (150, 0, 7, 0), (215, 7, 8, 0)]  # slots reused: other positions
    xp, xs, xd, rs, nd = [], [], [], [], []
    for p, sl, n, dn in rows:
        rs.append(len(xp))
        nd.append(n)
        for i in range(n + 1):
            xp.append(p + i)
            xs.append(sl)
            xd.append(dn if i == 0 else 0)
    T = len(xp) + 5  # unused tail pseudo-rows: done
    xp += [0] * 5
    xs += [0] * 5
    xd += [1] * 5
    i32 = dict(dtype=torch.int32, device=DEV)
    nd = [-1 if row[3] else n for row, n in zip(rows, nd)]  # finished rows: row_nd = -1 (sg_spec_plan)
    xp, xs, xd, rs, nd = (torch.tensor(v, **i32) for v in (xp, xs, xd, rs, nd))
    # the grouped kernel skips only the row's FIRST pseudo-row on done; mark its drafts done too
    xd_g = xd.clone()
    for r, (p, sl, n, dn) in enumerate(rows):
        if dn:
            xd_g[int(rs[r]):int(rs[r]) + n + 1] = 1
    q = _bf(T, nh, D, seed=24)
    scale = 1 / math.sqrt(D)
    out_s = torch.full((T, nh * D), 7.0, dtype=torch.bfloat16, device=DEV)
    out_g = out_s.clone()
    ops.attn_spec(q, rs, nd, xp, xs, xd, kc, vt, pk, pvt, P0, out_s, scale, max_q=max_q)
    ops.attn_decode(q, xp, xs, kc, vt, pk, pvt, P0, out_g, scale, done=xd_g, impl="grouped")
    torch.cuda.synchronize()
    assert torch.equal(out_s, out_g)
    for t in range(T):
        if int(xd_g[t]):
            assert torch.all(out_s[t] == 7.0)
            continue
        p, r = int(xp[t]), int(xs[t])
        ref = _ref_seq_attention(q[t:t + 1].float(), kc[r, :, :p + 1].permute(1, 0, 2).float(),
                                 vrows[r, :, :p + 1].permute(1, 0, 2).float(), pk[:, :P0].permute(1, 0, 2).float(),
                                 pvrows[:, :P0].permute(1, 0, 2).float(), P0, [p], scale)
        torch.testing.assert_close(out_s[t].float().view(1, nh, D), ref, atol=2e-2, rtol=2e-2)
    with pytest.raises(ValueError):
        ops.attn_spec(q, rs, nd, xp, xs, xd, kc, vt, pk, pvt, P0, out_s, scale, max_q=11)


# ---------------------------------------------------------------- operating points
# The headline bench runs the GEMMs at thousands of rows (decode halves of 4096 rows
# plus their drafts: ~9 216 pseudo-rows; prefill halves up to 16 384 tokens).  The
# kernels' multi-tile paths only run there: cfg 20 (persistent 256x256 SwiGLU) walks
# several tiles per block only once T > 256 tiles, i.e. from ~6 144 rows on.

@pytest.mark.parametrize("M", [6144, 9216, 16384])
@pytest.mark.parametrize("producer", [False, True])
def test_gemm_swiglu_persistent_operating_points(M, producer):
    """cfg 20 at bench-scale row counts: the persistent path that stages the next tile's
    first K-tile (and x² partials) inside the current tile's last K-tile, vs the fp32
    reference and vs the one-tile-per-block 128x128 kernel."""
    K, I = 576, 1536
    a = _bf(M, K, seed=71)
    gu = _bf(2 * I, K, scale=K ** -0.5, seed=72)
    nw = _bf(K, scale=0.1, seed=73) + 1
    w = ops.interleave_gate_up(ops.fold_norm(gu, nw))
    ss = None
    if producer:  # the partials a residual GEMM would write (NORM 2)
        ss = ops.ss_buffer(M, DEV)
        parts = a.float().pow(2).reshape(M, 9, 64).sum(-1).t()
        ss[:9, :M] = parts
    out = ops.gemm(a, w, epi="swiglu", norm_eps=1e-5, cfg=20, ss_in=ss)
    assert ops.gemm_cfg(M, 2 * I, epi="swiglu", K=K) == 20  # what the engine launches at these rows
    ref = ops.ref_gemm(a, gu, epi="swiglu", norm_eps=1e-5, norm_w=nw)
    rows = torch.randperm(M, generator=torch.Generator().manual_seed(M))[:512].to(DEV)  # fp32 reference on a sample
    torch.testing.assert_close(out.float()[rows], ref[rows], atol=3e-2, rtol=3e-2)
    base = ops.gemm(a, w, epi="swiglu", norm_eps=1e-5, cfg=0, ss_in=ss)
    torch.testing.assert_close(out.float(), base.float(), atol=2e-2, rtol=2e-2)


def _measured_cases():
    out = []
    for (epi, N, K), ranges in sorted(ops.GEMM_MEASURED.items()):
        for lo, hi, cfg in ranges:
            out.append((epi, N, K, cfg, min(hi, (lo + hi) // 2 if hi < (1 << 20) else lo + 2048)))
    return out


@pytest.mark.parametrize("epi,N,K,cfg,M", _measured_cases())
def test_gemm_measured_exceptions_in_range(epi, N, K, cfg, M):
    """Every tile exception of ops.GEMM_MEASURED at a row count inside its measured
    range (the configuration the engine really launches there) vs fp32."""
    assert ops.gemm_cfg(M, N, epi=epi, K=K) == cfg
    a = _bf(M, K, seed=81)
    if epi == "swiglu":
        gu = _bf(N, K, scale=K ** -0.5, seed=82)
        nw = _bf(K, scale=0.1, seed=83) + 1
        out = ops.gemm(a, ops.interleave_gate_up(ops.fold_norm(gu, nw)), epi="swiglu", norm_eps=1e-5)
        ref = ops.ref_gemm(a, gu, epi="swiglu", norm_eps=1e-5, norm_w=nw)
    else:
        w = _bf(N, K, scale=K ** -0.5, seed=84)
        x = _bf(M, N, seed=85)
        ref = x.float() + (a.float() @ w.float().t()).to(torch.bfloat16).float()
        out = ops.gemm(a, w, epi="resid", resid=x)
    rows = torch.randperm(M, generator=torch.Generator().manual_seed(M))[:512].to(DEV)
    torch.testing.assert_close(out.float()[rows], ref[rows], atol=3e-2, rtol=3e-2)


def test_attn_spec_bench_scale():
    """Verify attention at a bench-scale bucket: 4 096 rows, up to 6 drafts each
    (max_q 7, two MFMA column blocks), random positions over the whole slot, a
    quarter of the rows finished -- bit-identical to the grouped decode kernel on
    the same pseudo-rows, and an fp32 spot check."""
    nh, nkv, D, S, Lmax, P0 = 9, 3, 64, 4096, 224, 20
    P0pad = 32
    g = torch.Generator(device="cpu").manual_seed(91)
    kc = _bf(S, nkv, Lmax, D, seed=92)
    vrows = _bf(S, nkv, Lmax, D, seed=93)
    vt = ops.rows_to_vt(vrows)
    pk = torch.zeros(nkv, P0pad, D, dtype=torch.bfloat16, device=DEV)
    pvrows = torch.zeros(nkv, P0pad, D, dtype=torch.bfloat16, device=DEV)
    pk[:, :P0] = _bf(nkv, P0, D, seed=94)
    pvrows[:, :P0] = _bf(nkv, P0, D, seed=95)
    pvt = ops.rows_to_vt(pvrows)
    B, max_q = 4096, 7
    nd_h = torch.randint(0, max_q, (B,), generator=g)
    pos_h = torch.randint(0, Lmax - max_q, (B,), generator=g)
    done_h = torch.rand(B, generator=g) < 0.25
    slots = torch.randperm(S, generator=g)[:B]
    xp, xs, xd, rs, nd = [], [], [], [], []
    for r in range(B):
        rs.append(len(xp))
        if done_h[r]:
            nd.append(-1)
            continue
        nd.append(int(nd_h[r]))
        for i in range(int(nd_h[r]) + 1):
            xp.append(int(pos_h[r]) + i)
            xs.append(int(slots[r]))
            xd.append(0)
    T = len(xp)
    i32 = dict(dtype=torch.int32, device=DEV)
    xp, xs, xd, rs, nd = (torch.tensor(v, **i32) for v in (xp, xs, xd, rs, nd))
    q = _bf(T, nh, D, seed=96)
    scale = 1 / math.sqrt(D)
    out_s = torch.zeros(T, nh * D, dtype=torch.bfloat16, device=DEV)
    out_g = torch.zeros_like(out_s)
    ops.attn_spec(q, rs, nd, xp, xs, xd, kc, vt, pk, pvt, P0, out_s, scale, max_q=max_q)
    ops.attn_decode(q, xp, xs, kc, vt, pk, pvt, P0, out_g, scale, done=xd, impl="grouped")
    torch.cuda.synchronize()
    assert torch.equal(out_s, out_g)
    for t in torch.randperm(T, generator=g)[:24].tolist():
        p, r = int(xp[t]), int(xs[t])
        ref = _ref_seq_attention(q[t:t + 1].float(), kc[r, :, :p + 1].permute(1, 0, 2).float(),
                                 vrows[r, :, :p + 1].permute(1, 0, 2).float(), pk[:, :P0].permute(1, 0, 2).float(),
                                 pvrows[:, :P0].permute(1, 0, 2).float(), P0, [p], scale)
        torch.testing.assert_close(out_s[t].float().view(1, nh, D), ref, atol=2e-2, rtol=2e-2)


def test_kv_copy_prefix():
    """Template reuse copy: own offsets 0..k-1 of the template slot's keys, and the Vᵀ
    blocks holding them, land in the message slot on every layer; nothing else moves."""
    L, S, nkv, Lmax, D = 3, 10, 3, 64, 64
    kc = _bf(L, S, nkv, Lmax, D, seed=101)
    vt = _bf(L, *ops.vt_shape(S, nkv, D, Lmax), seed=102)
    k0, v0 = kc.clone(), vt.clone()
    items = torch.tensor([[8, 9, 8], [1, 4, 6], [5, 12, 1]], dtype=torch.int32, device=DEV)  # (src, dst, k)
    ops.kv_copy_prefix(kc, vt, items)
    torch.cuda.synchronize()
    ek, ev = k0.clone(), v0.clone()
    for src, dst, k in items.t().tolist():
        ek[:, dst, :, :k] = k0[:, src, :, :k]
        ev[:, dst, :, :(k + 7) // 8] = v0[:, src, :, :(k + 7) // 8]
    assert torch.equal(kc, ek) and torch.equal(vt, ev)


@pytest.mark.parametrize("M", [777, 9216])
def test_gemm_qkv_rope_tile_independent(M):
    """ops.qkv_cfg picks the QKV+RoPE tile by row count; every config accumulates each
    output in the same K order, so q, K and V^T come out bit-identical whatever the tile
    (a row's result never depends on the batch it runs in)."""
    nh, nkv, D, S, Lmax, K, p0 = 9, 3, 64, max(1024, M), 192, 576, 4
    x = _bf(M, K, seed=57)
    w = _bf((nh + 2 * nkv) * D, K, scale=K ** -0.5, seed=58)
    g = torch.Generator(device="cpu").manual_seed(59)
    pos = torch.randint(0, Lmax, (M,), generator=g, dtype=torch.int32).to(DEV)
    slot = torch.randperm(S, generator=g)[:M].to(torch.int32).to(DEV)
    cs = ops.rope_table(p0 + Lmax + 1, D, 100000.0, DEV)
    outs = []
    for cfg in (1, 3, 17, 23, 28):
        kc = torch.zeros(S, nkv, Lmax, D, dtype=torch.bfloat16, device=DEV)
        vt = torch.zeros(*ops.vt_shape(S, nkv, D, Lmax), dtype=torch.bfloat16, device=DEV)
        q = torch.zeros(M, nh, D, dtype=torch.bfloat16, device=DEV)
        ops.gemm_qkv_rope(x, w, 1e-5, pos, slot, cs, q, kc, vt, nh, nkv, p0, cfg=cfg)
        outs.append((q, kc, vt))
    for o in outs[1:]:
        for u, v in zip(outs[0], o):
            assert torch.equal(u, v)


def test_embed_rows_matches_f_embedding():
    """ops.embed_rows (int32 ids, one kernel) == F.embedding; ids outside the table -> 0."""
    import torch.nn.functional as F

    table = _bf(8192, 576, seed=91)
    ids = torch.randint(0, 8192, (9216,), dtype=torch.int32, device=DEV)
    assert torch.equal(ops.embed_rows(ids, table), F.embedding(ids.long(), table))
    bad = torch.tensor([-1, 8192, 5], dtype=torch.int32, device=DEV)
    out = ops.embed_rows(bad, table)
    assert torch.count_nonzero(out[:2]) == 0 and torch.equal(out[2], table[5])


@pytest.mark.parametrize("cfg", sorted(ops.GEMM_RESID_ONLY))
@pytest.mark.parametrize("M,K", [(110592, 1536), (55296, 576), (4099, 576)])
def test_gemm_resid_persistent_matches_cfg28(cfg, M, K):
    """The persistent staggered residual GEMM at the qa engine's operating points (many
    tiles per block: the step ring runs across tile boundaries): 16x16x32 (35 / 36)
    bit-identical to cfg 28, outputs and x² partials (the consumer's row scales do not
    depend on the config); 32x32x16 (37 / 38: other fp32 accumulation chunks) within
    rounding of it, partials within fp32 rounding."""
    H = 576
    a = _bf(M, K, seed=81)
    w = _bf(H, K, scale=K ** -0.5, seed=82)
    x = _bf(M, H, seed=83)
    x28, ss28 = x.clone(), ops.ss_buffer(M, DEV)
    ops.gemm(a, w, epi="resid", resid=x28, cfg=28, ss_out=ss28)
    xn, ssn = x.clone(), ops.ss_buffer(M, DEV)
    ops.gemm(a, w, epi="resid", resid=xn, cfg=cfg, ss_out=ssn)
    if cfg in (35, 36):
        assert torch.equal(xn, x28) and torch.equal(ssn, ss28)
    else:
        torch.testing.assert_close(xn.float(), x28.float(), atol=2e-2, rtol=1e-2)
        torch.testing.assert_close(ssn, ss28, rtol=2e-2, atol=1e-2)


@pytest.mark.parametrize("M", [77, 4099, 110592])
def test_gemm_swiglu_two_a_sets_match_cfg20(M):
    """cfg 42 (cfg 20 keeping both A register sets: p4 reads no LDS) issues the same
    MFMAs in the same order, so its SwiGLU output is bit-identical to cfg 20's."""
    H, I = 576, 1536
    x = _bf(M, H, seed=91)
    w = _bf(2 * I, H, scale=H ** -0.5, seed=92)
    ss = ops.ss_buffer(M, DEV)
    ss[:9, :M] = torch.rand(9, M, device=DEV)
    o20 = ops.gemm(x, w, epi="swiglu", norm_eps=1e-5, cfg=20, ss_in=ss)
    o42 = ops.gemm(x, w, epi="swiglu", norm_eps=1e-5, cfg=42, ss_in=ss)
    assert torch.equal(o42, o20)


@pytest.mark.parametrize("M", [77, 1000, 9216, 70001])
def test_gemm_qk_rope_persistent_matches_cfg28(M):
    """cfg 39 (q / k heads through the persistent staggered 256x256 kernel, W rows loaded
    in the RoPE-pair order, rotation in registers; v heads through cfg 28) writes the
    same q rows and caches as cfg 28 -- V^T exactly, q / k to the last bf16 rounding
    (the row scales sum the producer's partials in another order) -- on packed
    sequences, with the producer's x² partials (NORM 2) and without (NORM 1)."""
    nh, nkv, D, Lmax, K, p0 = 9, 3, 64, 192, 576, 20
    g = torch.Generator(device="cpu").manual_seed(71)
    lens = []
    while sum(lens) < M:
        lens.append(int(torch.randint(1, 71, (1,), generator=g)))
    lens[-1] -= sum(lens) - M
    lens = [n for n in lens if n > 0]
    S = len(lens)
    pos = torch.cat([torch.arange(n) for n in lens]).to(torch.int32).to(DEV)
    slot = torch.repeat_interleave(torch.randperm(S, generator=g), torch.tensor(lens)).to(torch.int32).to(DEV)
    a = _bf(M, K, seed=72)
    wo = _bf(K, K, scale=K ** -0.5, seed=73)
    x = _bf(M, K, seed=74)
    ss = ops.ss_buffer((M + 3) // 4 * 4, DEV)
    ops.gemm(a, wo, epi="resid", resid=x, cfg=28, ss_out=ss)  # x and its rows' x² partials
    w = _bf((nh + 2 * nkv) * D, K, scale=K ** -0.5, seed=75)
    cs = ops.rope_table(p0 + Lmax + 1, D, 100000.0, DEV)
    for ss_in in (ss, None):
        outs = []
        for cfg in (28, 39):
            kc = torch.zeros(S, nkv, Lmax, D, dtype=torch.bfloat16, device=DEV)
            vt = torch.zeros(*ops.vt_shape(S, nkv, D, Lmax), dtype=torch.bfloat16, device=DEV)
            q = torch.zeros(M, nh, D, dtype=torch.bfloat16, device=DEV)
            ops.gemm_qkv_rope(x, w, 1e-5, pos, slot, cs, q, kc, vt, nh, nkv, p0, cfg=cfg, ss_in=ss_in)
            outs.append((q, kc, vt))
        (q28, k28, v28), (q39, k39, v39) = outs
        assert torch.equal(v39, v28)
        for u, v in ((q39, q28), (k39, k28)):
            torch.testing.assert_close(u.float(), v.float(), atol=1e-2, rtol=1e-2)
            assert (u == v).float().mean() > 0.98, (u != v).float().mean()
