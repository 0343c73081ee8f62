"""TEST INFRASTRUCTURE (oracle): the reference's he::math / he::util schedules restated over the oracle's SEAL 4.1
Evaluator (oracle_py.Oracle), to check the GPU drop-in (cpp/src/he_math.cpp, cpp/include/he_util.h) bit for bit.
Never imported by the product.

Every function issues the reference's sequence of scalar encodes (CKKSEncoder::encode(double, parms_id, scale),
Oracle.encode_scalar), plaintext / ciphertext products, relinearizations and rescales; file:line per function.
Parity against SEAL itself is unpinned (no SEAL here, no reference vectors)."""
import math

import numpy as np


def _times_const(o, ct, c):
    """ct (x) encode(c, ct.parms_id, ct.scale), rescaled"""
    return o.rescale(o.multiply_plain(ct, o.encode_scalar(c, ct.scale, ct.level), ct.scale))


def _times_ct(o, rk, a, b=None):
    """rescale(relin(a * b)); b None squares"""
    return o.rescale(o.relinearize(o.square(a) if b is None else o.multiply(a, b), rk))


def drop_chain_levels(o, cts, num_of_levels):
    """he_util.h:27-48: per level, 1 encoded once at the first ciphertext's parms_id and scale, then multiply_plain +
    rescale_to_next of every ciphertext"""
    cts = list(cts)
    for _ in range(num_of_levels):
        one, sc = o.encode_scalar(1.0, cts[0].scale, cts[0].level), cts[0].scale
        cts = [o.rescale(o.multiply_plain(c, one, sc)) for c in cts]
    return cts


def reach_chain_level(o, cts, to_reach):
    """he_util.h:57-70: chain index = level - 1, so the levels to drop are the level difference"""
    return drop_chain_levels(o, cts, cts[0].level - to_reach.level)


def signed_inv(o, rk, x, a, iter_num):
    """he_math.cpp:22-90"""
    y = o.rescale(o.multiply_plain(x, o.encode_scalar(-a * a, x.scale, x.level), x.scale))
    y = o.add_plain(y, o.encode_scalar(2 * a, y.scale, y.level), y.scale)
    if iter_num == 1:
        return y
    e = o.rescale(o.multiply_plain(x, o.encode_scalar(a, x.scale, x.level), x.scale))
    one, one_scale = o.encode_scalar(1.0, e.scale, e.level), e.scale
    e = o.sub_plain(e, one, one_scale)
    y = o.rescale(o.multiply_plain(y, one, one_scale))
    for _ in range(1, iter_num):
        e = _times_ct(o, rk, e)
        term = o.add_plain(e, o.encode_scalar(1.0, e.scale, e.level), e.scale)
        y = _times_ct(o, rk, y, term)
    return y


def inv_sqrt_twice(o, rk, x, a, iter_num):
    """he_math.cpp:95-164 (the `#if 1` branch)"""
    y0 = a
    y = o.rescale(o.multiply_plain(x, o.encode_scalar(-y0 * y0 * y0, x.scale, x.level), x.scale))
    y = o.add_plain(y, o.encode_scalar(3.0 / 2 * y0, y.scale, y.level), y.scale)
    for i in range(1, iter_num):
        yp = y.copy()
        y = _times_const(o, y, 3.0 / 2)
        y = _times_const(o, y, 1.0)
        for _ in range(2 if i > 1 else 1):
            x = _times_const(o, x, 1.0)
        xy = _times_ct(o, rk, x, yp)
        yp = _times_ct(o, rk, yp)
        yp = _times_ct(o, rk, yp, xy)
        y = o.sub(y, yp)
    return y


def sqrt(o, rk, x, a, iter_num):
    """he_math.cpp:211-232"""
    y = inv_sqrt_twice(o, rk, x, 1 / a / math.sqrt(2), iter_num)
    s = o.rescale(o.multiply_plain(x, o.encode_scalar(math.sqrt(2), x.scale, x.level), x.scale))
    (s,) = reach_chain_level(o, [s], y)
    return _times_ct(o, rk, y, s)


def abs_(o, rk, x, a, iter_num):
    """he_math.cpp:237-269"""
    sq = _times_ct(o, rk, x)
    y = inv_sqrt_twice(o, rk, sq, 1 / a / math.sqrt(2), iter_num)
    sq = _times_const(o, sq, math.sqrt(2))
    for _ in range(sq.level - y.level):
        sq = _times_const(o, sq, 1.0)
    return _times_ct(o, rk, y, sq)


def least_squares_2d(o, rk, gk, x_ct, y_ct, n):
    """matrix_operations.cpp:915-1003 (bench_he_least_squares_2d after encryption): the sums of x, y, x^2, x y over the
    n data slots, the denominator n sum(x^2) - sum(x)^2 and its inverse by signed_inv(0.05, 6), the numerators of a and
    b, and a, b.  Returns [denom, denom_inv, a_num, b_num, a, b]."""
    sum_x = o.sum_elems(x_ct, n, gk)
    sum_y = o.sum_elems(y_ct, n, gk)
    sq = o.rescale(o.relinearize(o.square(x_ct), rk))                # BatchedVector::square (he_linalg.cpp:657-662)
    sum_xx = o.sum_elems(sq, n, gk)
    xy = o.rescale(o.relinearize(o.multiply(x_ct, y_ct), rk))        # eval % rk % x_ctv * y_ctv
    sum_xy = o.sum_elems(xy, n, gk)
    n_pt, n_scale = o.encode_scalar(float(n), sum_xx.scale, sum_xx.level), sum_xx.scale
    n_sum_xx = o.rescale(o.multiply_plain(sum_xx, n_pt, n_scale))
    sum_x_sqr = _times_ct(o, rk, sum_x)
    one, one_scale = o.encode_scalar(1.0, sum_x_sqr.scale, sum_x_sqr.level), sum_x_sqr.scale
    sum_x_sqr = o.rescale(o.multiply_plain(sum_x_sqr, one, one_scale))
    denom = o.sub(n_sum_xx, sum_x_sqr)
    one_v = o.encode(np.array([1.0]), denom.scale, denom.level)      # encode(vector<double>{1}, parms_id, scale)
    denom = o.rescale(o.multiply_plain(denom, one_v, denom.scale))
    denom_inv = signed_inv(o, rk, denom, 0.05, 6)
    n_sum_xy = o.rescale(o.multiply_plain(sum_xy, n_pt, n_scale))
    sxsy = _times_ct(o, rk, sum_x, sum_y)
    sxsy = o.rescale(o.multiply_plain(sxsy, one, one_scale))
    a_num = o.sub(n_sum_xy, sxsy)
    one, one_scale = o.encode_scalar(1.0, sum_y.scale, sum_y.level), sum_y.scale
    sysxx = o.rescale(o.multiply_plain(sum_y, one, one_scale))
    sysxx = _times_ct(o, rk, sysxx, sum_xx)
    sxsxy = o.rescale(o.multiply_plain(sum_x, one, one_scale))
    sxsxy = _times_ct(o, rk, sxsxy, sum_xy)
    b_num = o.sub(sysxx, sxsxy)
    a_num, b_num = reach_chain_level(o, [a_num, b_num], denom_inv)
    return [denom, denom_inv, a_num, b_num, _times_ct(o, rk, a_num, denom_inv), _times_ct(o, rk, b_num, denom_inv)]
