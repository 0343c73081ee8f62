#pragma once
// Drop-in for the reference's he::math (include/he_math.h:6-34) over hecdna types: Newton / Goldschmidt iterations
// for 1/x, 1/sqrt(2x), sqrt(x) and |x| on CKKS ciphertexts.  Each function issues the reference's sequence of
// scalar encodes, plaintext and ciphertext products, relinearizations and rescales (src/core/he_math.cpp:22-269),
// so on the same inputs and keys every intermediate ciphertext equals SEAL's bit for bit.
#include <cstddef>

#include "he_operators.h"
#include "hecdna/seal_compat.hpp"

namespace he::math
{
    // f(x) = 1/x; a predicts the result with |a x - 1| < 1 (he_math.h:8-15)
    hecdna::Ciphertext signed_inv(const hecdna::CKKSEncoder &cencd, const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk,
                                  const hecdna::Ciphertext &x_ct, double a, std::size_t iter_num);

    // f(x) = 1/sqrt(2x), x > 0; 0 < a < sqrt(3/(2x)) (he_math.h:17-23)
    hecdna::Ciphertext inv_sqrt_twice(const hecdna::CKKSEncoder &cencd, const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk,
                                      const hecdna::Ciphertext &x_ct, double a, std::size_t iter_num);

    // f(x) = sqrt(x) (he_math.h:25-28)
    hecdna::Ciphertext sqrt(const hecdna::Context &ctx, const hecdna::CKKSEncoder &cencd, const hecdna::Evaluator &eval,
                            const hecdna::RelinKeys &rk, const hecdna::Ciphertext &x_ct, double a, std::size_t iter_num);

    // f(x) = |x| (he_math.h:30-33)
    hecdna::Ciphertext abs(const hecdna::Context &ctx, const hecdna::CKKSEncoder &cencd, const hecdna::Evaluator &eval,
                           const hecdna::RelinKeys &rk, const hecdna::Ciphertext &x_ct, double a, std::size_t iter_num);
} // namespace he::math
