"""Sampled stage timing (dg_encode_plan_set_timing_every,
dg_decode_plan_set_timing_every): bench.py records the kernel events on every
4th timed step only.  The runs with and without events must produce the same
bytes, the ring must hold only recorded runs, and the stage times must be
positive; an invalid stride is refused."""
import pytest

pytestmark = pytest.mark.gpu


def test_encode_timing_every(dg, ctx, orc, torch_cuda):
    torch = torch_cuda
    n, L = 64, 16384
    ref = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    ver = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    ctx.check(dg.lib.dg_synth_edit_pairs_device(ctx.handle, ref.data_ptr(), ver.data_ptr(), n, L,
                                                7, 160, None), "synth")
    plan = dg.EncodePlan(ctx, "onepass", [(i * L, L, i * L, L) for i in range(n)], q=1)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    run = lambda: plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(),
                           off.data_ptr(), st.data_ptr(), ctx.stream)
    torch.cuda.synchronize()
    run()
    torch.cuda.synchronize()
    want = bytes(out[: int(off[-1])].cpu().numpy())
    assert int((st != 0).sum()) == 0
    for dominant in (False, True):
        plan.set_timing(2, dominant_only=dominant, every=3)
        for k in range(7):   # runs 0, 3, 6 record; the ring keeps 3 and 6
            out.zero_()
            run()
            torch.cuda.synchronize()
            assert bytes(out[: int(off[-1])].cpu().numpy()) == want, (dominant, k)
        t = plan.stage_times()
        assert t.get("diff", 0) > 0, t
    plan.set_timing(0)
    with pytest.raises(Exception):
        plan.set_timing(1, every=0)
    R, V = bytes(ref[:L].cpu().numpy()), bytes(ver[:L].cpu().numpy())
    assert want[: int(off[1])] == orc.encode(1, R, V, p=16, q=1)


def test_decode_timing_every(dg, ctx, orc, torch_cuda):
    torch = torch_cuda
    import random
    rng = random.Random(5)
    items = []
    for _ in range(8):
        R = rng.randbytes(20000)
        V = R[:7000] + rng.randbytes(300) + R[7000:]
        items.append((R, orc.encode(1, R, V, p=16, q=1), V))
    up = lambda x: (x + 15) // 16 * 16
    descs, ro, do, oo = [], 0, 0, 0
    for R, d, V in items:
        descs.append((ro, len(R), do, len(d), oo, len(V)))
        ro += up(len(R)); do += len(d); oo += up(len(V))
    ref = torch.zeros(ro, dtype=torch.uint8)
    dl = torch.zeros(max(do, 16), dtype=torch.uint8)
    for (R, d, _), (r0, _, d0, _, _, _) in zip(items, descs):
        ref[r0:r0 + len(R)] = torch.frombuffer(bytearray(R), dtype=torch.uint8)
        dl[d0:d0 + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8)
    ref, dl = ref.cuda(), dl.cuda()
    out = torch.zeros(oo, dtype=torch.uint8, device="cuda")
    olen = torch.zeros(len(items), dtype=torch.int64, device="cuda")
    st = torch.zeros(len(items), dtype=torch.int32, device="cuda")
    plan = dg.DecodePlan(ctx, descs)
    plan.set_timing(2, every=2)
    for _ in range(5):   # runs 0, 2, 4 record
        out.zero_()
        torch.cuda.synchronize()
        plan.run(ref.data_ptr(), dl.data_ptr(), out.data_ptr(), olen.data_ptr(), st.data_ptr(), ctx.stream)
        torch.cuda.synchronize()
        assert st.cpu().tolist() == [0] * len(items)
        oc = out.cpu()
        for (R, d, V), ds in zip(items, descs):
            assert bytes(oc[ds[4]:ds[4] + len(V)].numpy()) == V
    t = plan.stage_times()
    assert list(t) == ["decode"] and t["decode"] > 0, t
    with pytest.raises(Exception):
        plan.set_timing(1, every=0)
