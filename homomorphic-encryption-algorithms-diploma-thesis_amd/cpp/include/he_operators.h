#pragma once
// Drop-in for the reference's he::operators (include/he_operators.h:13-159): the same tie operator
// `%` and the same operator overloads, declared over hecdna types instead of seal:: types.  Each
// operator forwards 1:1 to the hecdna::Evaluator member that replaces the seal::Evaluator call of
// the reference (src/core/he_operators.cpp:14-237).
#include <concepts>
#include <tuple>
#include <type_traits>
#include <utility>

#include "hecdna/seal_compat.hpp"

namespace he::operators
{
    template <typename T>
    concept Plaintext_Ciphertext_GaloisKeys_RelinKeys_tn = std::same_as<std::decay_t<T>, hecdna::Plaintext> ||
                                                           std::same_as<std::decay_t<T>, hecdna::Ciphertext> ||
                                                           std::same_as<std::decay_t<T>, hecdna::GaloisKeys> ||
                                                           std::same_as<std::decay_t<T>, hecdna::RelinKeys>;

    // eval % x  (he_operators.h:22-27)
    template <Plaintext_Ciphertext_GaloisKeys_RelinKeys_tn T>
    constexpr auto operator%(const hecdna::Evaluator &eval, T &&op)
    {
        return std::tie(eval, std::forward<T>(op));
    }

    template <typename T>
    concept Ciphertext_int_tn = std::same_as<std::decay_t<T>, hecdna::Ciphertext> || std::same_as<std::decay_t<T>, int>;

    // eval % gk % x  (he_operators.h:35-39)
    template <Ciphertext_int_tn T>
    constexpr auto operator%(const std::tuple<const hecdna::Evaluator &, const hecdna::GaloisKeys &> &eval_gk, T &&op)
    {
        return std::tie(eval_gk, std::forward<T>(op));
    }

    using EvalCt = std::tuple<const hecdna::Evaluator &, const hecdna::Ciphertext &>;
    using EvalPt = std::tuple<const hecdna::Evaluator &, const hecdna::Plaintext &>;
    using EvalRk = std::tuple<const hecdna::Evaluator &, const hecdna::RelinKeys &>;
    using EvalGk = std::tuple<const hecdna::Evaluator &, const hecdna::GaloisKeys &>;

    hecdna::Ciphertext &operator-=(hecdna::Ciphertext &op, const hecdna::Evaluator &eval);        // negate
    hecdna::Ciphertext operator-(const EvalCt &eval_op);
    hecdna::Ciphertext &operator+=(hecdna::Ciphertext &op1, const EvalCt &eval_op2);               // add
    hecdna::Ciphertext operator+(const EvalCt &eval_op1, const hecdna::Ciphertext &op2);
    hecdna::Ciphertext &operator+=(hecdna::Ciphertext &op1, const EvalPt &eval_op2);               // add plain
    hecdna::Ciphertext operator+(const EvalCt &eval_op1, const hecdna::Plaintext &op2);
    hecdna::Ciphertext &operator-=(hecdna::Ciphertext &op1, const EvalCt &eval_op2);               // sub
    hecdna::Ciphertext operator-(const EvalCt &eval_op1, const hecdna::Ciphertext &op2);
    hecdna::Ciphertext &operator-=(hecdna::Ciphertext &op1, const EvalPt &eval_op2);               // sub plain
    hecdna::Ciphertext operator-(const EvalCt &eval_op1, const hecdna::Plaintext &op2);
    hecdna::Ciphertext &operator*=(hecdna::Ciphertext &op1, const EvalCt &eval_op2);               // multiply
    hecdna::Ciphertext operator*(const EvalCt &eval_op1, const hecdna::Ciphertext &op2);
    hecdna::Ciphertext &operator*=(hecdna::Ciphertext &op1, const EvalPt &eval_op2);               // multiply plain
    hecdna::Ciphertext operator*(const EvalCt &eval_op1, const hecdna::Plaintext &op2);
    hecdna::Ciphertext &operator&=(hecdna::Ciphertext &op, const EvalRk &eval_rk);                 // relinearize
    hecdna::Ciphertext operator&(const EvalRk &eval_rk, const hecdna::Ciphertext &op);
    hecdna::Ciphertext &operator^=(hecdna::Ciphertext &op, const hecdna::Evaluator &eval);        // rescale to next
    hecdna::Ciphertext operator^(const hecdna::Evaluator &eval, const hecdna::Ciphertext &op);
    hecdna::Ciphertext &operator|=(hecdna::Ciphertext &op, const hecdna::Evaluator &eval);        // mod switch to next
    hecdna::Ciphertext operator|(const hecdna::Evaluator &eval, const hecdna::Ciphertext &op);
    // rotate left / right (he_operators.h:144-159)
    hecdna::Ciphertext &operator<<=(hecdna::Ciphertext &op, const std::tuple<const EvalGk &, const int &> &eval_gk__steps);
    hecdna::Ciphertext operator<<(const std::tuple<const EvalGk &, const hecdna::Ciphertext &> &eval_gk__op, int steps);
    hecdna::Ciphertext &operator>>=(hecdna::Ciphertext &op, const std::tuple<const EvalGk &, const int &> &eval_gk__steps);
    hecdna::Ciphertext operator>>(const std::tuple<const EvalGk &, const hecdna::Ciphertext &> &eval_gk__op, int steps);
} // namespace he::operators
