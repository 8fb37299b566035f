"""The per-sample path's fast square roots and reciprocals (rr_device.h
sqrt_rn / sqrt_any / rcp_rn) return the bits of the device's correctly
rounded sqrtf and 1.0f / x — and so of the oracle's — for every float the
path passes them: checked here over all 2^32 bit patterns on the device
(rr_debug_fastmath_check)."""
import pytest

pytestmark = pytest.mark.gpu


def test_fast_sqrt_and_reciprocal_match_ieee_on_every_float(ctx):
    sq_in, sq_out, sq_any, rc_in, rc_out = ctx.fastmath_check(0, 1 << 32)
    print(f"sqrt_rn mismatches: {sq_in} in range, {sq_out} outside; sqrt_any: {sq_any}; "
          f"rcp_rn: {rc_in} in range, {rc_out} outside")
    assert sq_in == 0  # +-0 and [2^-96, FLT_MAX]: every call site of sqrt_rn stays in there
    assert sq_any == 0  # the guarded form is exact everywhere
    assert rc_in == 0  # |x| in [2^-126, 2^126): every call site of rcp_rn stays in there
    assert rc_out > 0  # subnormals, zero and |x| >= 2^126 need the division's wrappers
    assert sq_out > 0  # the range restriction is real (subnormals, tiny normals, inf)


def test_fastmath_check_arguments(ctx, rr):
    assert ctx.fastmath_check(0x3F800000, 1 << 20) == (0, 0, 0, 0, 0)  # [1, 1.125)
    with pytest.raises(rr.RRError):
        ctx.fastmath_check(0xFFFFFFFF, 2)  # past the last pattern
