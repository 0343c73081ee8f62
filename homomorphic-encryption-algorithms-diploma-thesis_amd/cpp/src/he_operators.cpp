// he::operators over hecdna (reference src/core/he_operators.cpp:14-237): every operator is a
// 1:1 call of the hecdna::Evaluator member replacing the seal::Evaluator call; out-of-place forms
// return a new value (value semantics, like the reference).
#include "he_operators.h"

using hecdna::Ciphertext;
using hecdna::Evaluator;
using std::get;

namespace he::operators
{
    Ciphertext &operator-=(Ciphertext &op, const Evaluator &eval) { eval.negate_inplace(op); return op; }
    Ciphertext operator-(const EvalCt &e) { Ciphertext r; get<0>(e).negate(get<1>(e), r); return r; }

    Ciphertext &operator+=(Ciphertext &a, const EvalCt &e) { get<0>(e).add_inplace(a, get<1>(e)); return a; }
    Ciphertext operator+(const EvalCt &e, const Ciphertext &b) { Ciphertext r; get<0>(e).add(get<1>(e), b, r); return r; }
    Ciphertext &operator+=(Ciphertext &a, const EvalPt &e) { get<0>(e).add_plain_inplace(a, get<1>(e)); return a; }
    Ciphertext operator+(const EvalCt &e, const hecdna::Plaintext &p)
    {
        Ciphertext r;
        get<0>(e).add_plain(get<1>(e), p, r);
        return r;
    }

    Ciphertext &operator-=(Ciphertext &a, const EvalCt &e) { get<0>(e).sub_inplace(a, get<1>(e)); return a; }
    Ciphertext operator-(const EvalCt &e, const Ciphertext &b) { Ciphertext r; get<0>(e).sub(get<1>(e), b, r); return r; }
    Ciphertext &operator-=(Ciphertext &a, const EvalPt &e) { get<0>(e).sub_plain_inplace(a, get<1>(e)); return a; }
    Ciphertext operator-(const EvalCt &e, const hecdna::Plaintext &p)
    {
        Ciphertext r;
        get<0>(e).sub_plain(get<1>(e), p, r);
        return r;
    }

    Ciphertext &operator*=(Ciphertext &a, const EvalCt &e) { get<0>(e).multiply_inplace(a, get<1>(e)); return a; }
    Ciphertext operator*(const EvalCt &e, const Ciphertext &b)
    {
        Ciphertext r;
        get<0>(e).multiply(get<1>(e), b, r);
        return r;
    }
    Ciphertext &operator*=(Ciphertext &a, const EvalPt &e) { get<0>(e).multiply_plain_inplace(a, get<1>(e)); return a; }
    Ciphertext operator*(const EvalCt &e, const hecdna::Plaintext &p)
    {
        Ciphertext r;
        get<0>(e).multiply_plain(get<1>(e), p, r);
        return r;
    }

    Ciphertext &operator&=(Ciphertext &a, const EvalRk &e) { get<0>(e).relinearize_inplace(a, get<1>(e)); return a; }
    Ciphertext operator&(const EvalRk &e, const Ciphertext &a)
    {
        Ciphertext r;
        get<0>(e).relinearize(a, get<1>(e), r);
        return r;
    }

    Ciphertext &operator^=(Ciphertext &a, const Evaluator &eval) { eval.rescale_to_next_inplace(a); return a; }
    Ciphertext operator^(const Evaluator &eval, const Ciphertext &a) { Ciphertext r; eval.rescale_to_next(a, r); return r; }
    Ciphertext &operator|=(Ciphertext &a, const Evaluator &eval) { eval.mod_switch_to_next_inplace(a); return a; }
    Ciphertext operator|(const Evaluator &eval, const Ciphertext &a) { Ciphertext r; eval.mod_switch_to_next(a, r); return r; }

    Ciphertext &operator<<=(Ciphertext &a, const std::tuple<const EvalGk &, const int &> &e)
    {
        get<0>(get<0>(e)).rotate_vector_inplace(a, get<1>(e), get<1>(get<0>(e)));
        return a;
    }
    Ciphertext operator<<(const std::tuple<const EvalGk &, const Ciphertext &> &e, int steps)
    {
        Ciphertext r;
        get<0>(get<0>(e)).rotate_vector(get<1>(e), steps, get<1>(get<0>(e)), r);
        return r;
    }
    Ciphertext &operator>>=(Ciphertext &a, const std::tuple<const EvalGk &, const int &> &e)
    {
        get<0>(get<0>(e)).rotate_vector_inplace(a, -get<1>(e), get<1>(get<0>(e)));
        return a;
    }
    Ciphertext operator>>(const std::tuple<const EvalGk &, const Ciphertext &> &e, int steps)
    {
        Ciphertext r;
        get<0>(get<0>(e)).rotate_vector(get<1>(e), -steps, get<1>(get<0>(e)), r);
        return r;
    }
} // namespace he::operators
