"""Band row strides (rifraf_hip.hip band_stride / rf_realign, mirrored by
rifraf_amd.bandedarrays.band_stride for arena sizing): a realign call whose
widest band reaches RF_OPT_BAND_PAD lays out every band with rows of whole
128-B lines (multiples of 16 doubles); other calls keep ceil(H/2) | 1."""
import numpy as np

from rifraf_amd.bandedarrays import BAND_PAD_H, band_stride


def test_band_stride_values():
    assert BAND_PAD_H == 64
    # c4-like calls (widest band below the threshold) keep the odd stride
    np.testing.assert_array_equal(band_stride(np.array([1, 2, 19, 20, 29, 31, 33, 63])),
                                  [1, 1, 11, 11, 15, 17, 17, 33])
    # a call with one wide band pads all of its bands
    np.testing.assert_array_equal(band_stride(np.array([19, 32, 37, 64, 65, 128, 129, 255])),
                                  [16, 16, 32, 32, 48, 64, 80, 128])
    H = np.arange(1, 600)
    P = band_stride(H)
    assert np.all(P % 16 == 0) and np.all(P >= (H + 1) // 2) and np.all(P - (H + 1) // 2 < 16)


def test_band_stride_option():
    assert band_stride(100, pad_h=0) == 51            # 0: odd stride everywhere
    assert band_stride(20, pad_h=1) == 16             # 1: every call padded
    np.testing.assert_array_equal(band_stride(np.array([31, 39]), pad_h=40), [17, 21])
