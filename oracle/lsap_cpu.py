"""TEST INFRASTRUCTURE ONLY (never imported by the product path).

CPU restatement of the linear sum assignment the reference's HungarianMatcher calls
(`scipy.optimize.linear_sum_assignment`, `src/models/detrpose/matcher.py:97`; scipy 1.15.3
here, a dependency that is not vendored in the reference). scipy's published algorithm is
the shortest augmenting path of Crouse (2016, "On implementing 2D rectangular assignment
algorithms"), run on float64 costs with the matrix transposed when it has more rows than
columns; the result is returned with the row indices ascending. This restatement follows
that algorithm step by step, including its tie-breaks (column scan order, preference for
an unassigned column among equal path costs), so that it reproduces scipy's indices on
tie-heavy integer matrices too (pinned against scipy itself in tests/test_criterion.py).
The HIP kernel (`csrc/criterion.hip`, `dp_hungarian_match`) follows this restatement.
"""
from __future__ import annotations

import math

import numpy as np


def lsap(cost) -> tuple[np.ndarray, np.ndarray]:
    c = np.asarray(cost, dtype=np.float64)
    nr, nc = c.shape
    if nr == 0 or nc == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    transpose = nc < nr
    if transpose:
        c = c.T
        nr, nc = nc, nr
    u = np.zeros(nr)
    v = np.zeros(nc)
    col4row = np.full(nr, -1, np.int64)
    row4col = np.full(nc, -1, np.int64)
    for cur in range(nr):
        spc = np.full(nc, math.inf)
        path = np.full(nc, -1, np.int64)
        SR = np.zeros(nr, bool)
        SC = np.zeros(nc, bool)
        remaining = [nc - it - 1 for it in range(nc)]
        num_rem = nc
        min_val = 0.0
        i = cur
        sink = -1
        while sink == -1:
            SR[i] = True
            lowest = math.inf
            index = -1
            for it in range(num_rem):
                j = remaining[it]
                r = min_val + c[i, j] - u[i] - v[j]
                if r < spc[j]:
                    path[j] = i
                    spc[j] = r
                if spc[j] < lowest or (spc[j] == lowest and row4col[j] == -1):
                    lowest = spc[j]
                    index = it
            min_val = lowest
            if min_val == math.inf:
                raise ValueError("cost matrix is infeasible")
            j = remaining[index]
            if row4col[j] == -1:
                sink = j
            else:
                i = row4col[j]
            SC[j] = True
            num_rem -= 1
            remaining[index] = remaining[num_rem]
        u[cur] += min_val
        for ii in range(nr):
            if SR[ii] and ii != cur:
                u[ii] += min_val - spc[col4row[ii]]
        for jj in range(nc):
            if SC[jj]:
                v[jj] -= min_val - spc[jj]
        j = sink
        while True:
            ii = path[j]
            row4col[j] = ii
            col4row[ii], j = j, col4row[ii]
            if ii == cur:
                break
    if transpose:
        order = np.argsort(col4row, kind="stable")
        return col4row[order], order.astype(np.int64)
    return np.arange(nr, dtype=np.int64), col4row
