"""The identity behind fp16_to_fixed24 (audio_rag_amd/csrc/armi_common.h): for every fp16 bit
pattern in the exact paths' domain (exponent field <= 15, |x| < 2), converting through fp32 --
float(x) * 2^24 truncated to int32 -- gives the same integer as the bit-field form
(mantissa | implicit bit) << (exponent - 1), negated for a set sign bit. The GPU code uses the
fp32 form (3 instructions); the int64 exact keys of the dense path rest on this equality."""

import numpy as np


def test_fp32_path_equals_bit_field_form_for_every_in_domain_fp16():
    h = np.arange(65536, dtype=np.uint32)
    e = (h >> 10) & 31
    dom = e <= 15
    m = h & 1023
    v = np.where(e == 0, m, (1024 | m) << np.maximum(e.astype(np.int64) - 1, 0)).astype(np.int64)
    v = np.where(h & 0x8000, -v, v)
    x = h[dom].astype(np.uint16).view(np.float16).astype(np.float32)
    f = (x * np.float32(16777216.0)).astype(np.int64)
    assert dom.sum() == 32768
    np.testing.assert_array_equal(f, v[dom])
    assert np.abs(f).max() < 2 ** 25
