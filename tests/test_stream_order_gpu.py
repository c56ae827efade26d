"""Stream ordering at the Python boundary (omr.Context(torch_order=True), the default): torch
kernels produce a call's inputs and consume its outputs with no explicit synchronize in
between; the context's non-blocking stream must wait for the former and torch for the latter.
A flip-mask test once read its output through torch before the context stream had finished."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rounds", [12])
def test_torch_produced_inputs_and_consumed_outputs(ctx, rounds):
    import torch
    w, h = 1024, 1024
    for i in range(rounds):
        src = torch.arange(w * h, dtype=torch.int32, device="cuda") * 7 + i      # torch kernels
        dst = torch.empty_like(src)
        ctx.flip_argb_device(src, dst, w, h, True, True)                        # context stream
        assert torch.equal(dst.flip(0), src), f"round {i}"                     # torch consumer
        m = (src & 0xFF).to(torch.uint8)
        md = torch.empty_like(m)
        ctx.flip_mask_device(m, md, w, h, True, False)
        assert torch.equal(md.view(h, w), m.view(h, w).flip(1)), f"mask round {i}"


def test_opt_out_context_needs_explicit_sync():
    """torch_order=False adds nothing to a call (the bench's contexts); after synchronize() the
    result is there."""
    import torch
    import omr
    with omr.Context(0, torch_order=False) as c:
        src = torch.arange(4096, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        dst = torch.empty_like(src)
        c.flip_argb_device(src, dst, 64, 64, True, True)
        c.synchronize()
        assert torch.equal(dst.flip(0), src)
