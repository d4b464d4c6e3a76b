"""BandedArray geometry (src/bandedarrays.jl:1-231).

On the engine a band lives in device memory in exactly the reference layout
(`data[(i-j)+h_off+bw+1, j]`, column-major, H = 2*bw + |nrows-ncols| + 1
data rows).  This host class carries the geometry and, when downloaded, the
data, so tests and host helpers can index it with the reference's 1-based
accessors.
"""
from __future__ import annotations

import numpy as np


def ndatarows(nrows: int, ncols: int, bandwidth: int) -> int:   # :101-104
    return 2 * bandwidth + abs(nrows - ncols) + 1


BAND_PAD_H = 64   # RF_OPT_BAND_PAD default (rifraf_hip.hip band_stride / rf_realign)


def band_stride(H, pad_h: int = BAND_PAD_H):
    """Row strides (doubles) of the device bands of ONE rf_realign call with
    band heights H: whole 128-B lines for every band when the call's widest
    band reaches pad_h (> 0; 1 = always), else the odd stride ceil(H/2) | 1."""
    H = np.asarray(H)
    half = (H + 1) >> 1
    pad = pad_h > 0 and H.size > 0 and int(H.max()) >= pad_h
    out = (half + 15) & ~15 if pad else half | 1
    return int(out) if out.ndim == 0 else out


def bandlimits(nrows: int, ncols: int, bandwidth: int):          # :44-53
    if ncols > nrows:
        return nrows - ncols - bandwidth, bandwidth
    return -bandwidth, nrows - ncols + bandwidth


def equal_ranges(a_range, b_range):                               # :220-231
    a_start, a_stop = a_range
    b_start, b_stop = b_range
    alen = a_stop - a_start + 1
    blen = b_stop - b_start + 1
    amin = max(b_start - a_start + 1, 1)
    amax = alen - max(a_stop - b_stop, 0)
    bmin = max(a_start - b_start + 1, 1)
    bmax = blen - max(b_stop - a_stop, 0)
    return (amin, amax), (bmin, bmax)


class BandedArray:
    """Sparse array with a band of non-zeroes (bandedarrays.jl:5-42)."""

    def __init__(self, shape, bandwidth: int, dtype=np.float64, default=0.0,
                 row_padding: int = 0, col_padding: int = 0, data=None):
        if bandwidth < 1:
            raise ValueError("bandwidth must be positive")
        self.dtype = dtype
        self.default = default
        self.row_padding = row_padding
        self.col_padding = col_padding
        self.bandwidth = int(bandwidth)
        self._set_shape(shape)
        if data is None:
            data = np.zeros((ndatarows(self.nrows, self.ncols, self.bandwidth) + row_padding,
                             self.ncols + col_padding), dtype=dtype, order="F")
        elif data.shape != (ndatarows(self.nrows, self.ncols, self.bandwidth) + row_padding,
                            self.ncols + col_padding):
            raise ValueError("data is wrong shape")
        self.data = data

    def _set_shape(self, shape):
        nrows, ncols = shape
        self.nrows, self.ncols = int(nrows), int(ncols)
        self.h_offset = max(self.ncols - self.nrows, 0)
        self.v_offset = max(self.nrows - self.ncols, 0)
        self.lower, self.upper = bandlimits(self.nrows, self.ncols, self.bandwidth)

    @property
    def shape(self):
        return (self.nrows, self.ncols)

    def resize(self, shape):                                      # :80-93
        self._set_shape(shape)
        drows, dcols = self.data.shape
        if ndatarows(self.nrows, self.ncols, self.bandwidth) > drows or self.ncols > dcols:
            self.reallocate()

    def newbandwidth(self, bandwidth: int):                       # :95-98
        self.bandwidth = int(bandwidth)
        self.lower, self.upper = bandlimits(self.nrows, self.ncols, self.bandwidth)
        self.reallocate()

    def reallocate(self):                                         # :74-78
        self.data = np.zeros((ndatarows(self.nrows, self.ncols, self.bandwidth) + self.row_padding,
                              self.ncols + self.col_padding), dtype=self.dtype, order="F")

    def inband(self, i: int, j: int) -> bool:                    # :151-157
        if i < 1 or j < 1 or i > self.nrows or j > self.ncols:
            return False
        return self.lower <= i - j <= self.upper

    def data_row(self, i: int, j: int) -> int:                   # :109-114
        if not self.inband(i, j):
            raise IndexError(f"[{i}, {j}] is not in band")
        return (i - j) + self.h_offset + self.bandwidth + 1

    def __getitem__(self, ij):                                    # :116-122
        i, j = ij
        if self.inband(i, j):
            return self.data[self.data_row(i, j) - 1, j - 1]
        return self.default

    def __setitem__(self, ij, v):                                 # :124-130
        i, j = ij
        if not self.inband(i, j):
            raise IndexError(f"Cannot set out-of-band element [{i}, {j}].")
        self.data[self.data_row(i, j) - 1, j - 1] = v

    def row_range(self, j: int):                                  # :133-137
        start = max(1, j - self.h_offset - self.bandwidth)
        stop = min(j + self.v_offset + self.bandwidth, self.nrows)
        return start, stop

    def data_row_range(self, j: int):                             # :140-143
        a, b = self.row_range(j)
        return self.data_row(a, j), self.data_row(b, j)

    def sparsecol(self, j: int):                                  # :146-149
        start, stop = self.data_row_range(j)
        return self.data[start - 1:stop, j - 1]

    def full(self):                                               # :160-168
        result = np.zeros((self.nrows, self.ncols), dtype=self.dtype)
        for j in range(1, self.ncols + 1):
            start, stop = self.row_range(j)
            dstart, dstop = self.data_row_range(j)
            result[start - 1:stop, j - 1] = self.data[dstart - 1:dstop, j - 1]
        return result

    def flip(self):                                               # :176-198
        nrows = ndatarows(self.nrows, self.ncols, self.bandwidth)
        a, b = divmod(self.ncols, 2)
        D = self.data
        for j in range(1, a + 1):
            for i in range(1, nrows + 1):
                D[i - 1, j - 1], D[nrows - i, self.ncols - j] = D[nrows - i, self.ncols - j], D[i - 1, j - 1]
        if b == 1:
            c = nrows // 2
            j = a + 1
            for i in range(1, c + 1):
                D[i - 1, j - 1], D[nrows - i, self.ncols - j] = D[nrows - i, self.ncols - j], D[i - 1, j - 1]

    def __repr__(self):
        return f"BandedArray(shape={self.shape}, bandwidth={self.bandwidth})"
