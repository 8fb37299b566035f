"""The per-sample path's fast square roots (rr_device.h sqrt_rn / sqrt_any)
return the bits of the device's correctly rounded sqrtf — and so of the
oracle's sqrtf — for every float the path passes them: checked here over all
2^32 bit patterns on the device (rr_debug_sqrt_check)."""
import pytest

pytestmark = pytest.mark.gpu


def test_sqrt_rn_matches_sqrtf_on_every_float(ctx):
    in_range, outside, any_ = ctx.sqrt_check(0, 1 << 32)
    print(f"sqrt_rn mismatches: {in_range} in range, {outside} outside; sqrt_any mismatches: {any_}")
    assert in_range == 0  # +-0 and [2^-96, FLT_MAX]: every call site of sqrt_rn stays in there
    assert any_ == 0      # the guarded form is exact everywhere
    assert outside > 0    # the range restriction is real (subnormals, tiny normals, inf)


def test_sqrt_check_arguments(ctx, rr):
    assert ctx.sqrt_check(0x3F800000, 1 << 20) == (0, 0, 0)  # [1, 1.125)
    with pytest.raises(rr.RRError):
        ctx.sqrt_check(0xFFFFFFFF, 2)  # past the last pattern
