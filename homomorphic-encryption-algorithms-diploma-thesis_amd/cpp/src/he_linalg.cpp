// he::linalg over hecdna — restates the reference's semantics (src/core/he_linalg.cpp) on the GPU
// engine.  Element-wise operations go through he::operators exactly like the reference; the two
// hot paths are single batched engine calls:
//   Matrix::matmul family      (:202-349) -> hec_matrix_matmul
//   BatchedMatrix::matmul      (:943-1006) -> hec_matmul_diag_col (diag x col) / hec_matmul_col_colT
#include "he_linalg.h"

#include <cassert>
#include <cmath>

using hecdna::Ciphertext;
using hecdna::Evaluator;
using hecdna::GaloisKeys;
using hecdna::RelinKeys;
using std::get;
using std::size_t;
using std::tuple;
using std::vector;
using namespace he::operators;  // as the reference does (he_linalg.cpp:6)

namespace he::linalg
{
    using he::operators::operator%;

    // =================================================================== Matrix
    Matrix::Matrix(size_t rows, size_t cols, const vector<Ciphertext> &e) : dims{rows, cols}, elems(e) {}
    Matrix::Matrix(size_t rows, size_t cols, vector<Ciphertext> &&e) : dims{rows, cols}, elems(std::move(e)) {}
    Matrix::Matrix(size_t rows, size_t cols) : Matrix(rows, cols, vector<Ciphertext>(rows * cols)) {}

    vector<size_t> Matrix::get_dims() const { return transposed ? vector<size_t>{dims[1], dims[0]} : dims; }
    bool Matrix::get_transp() const { return transposed; }
    void Matrix::transp() { transposed = !transposed; }
    const vector<Ciphertext> &Matrix::get_elems() const { return elems; }
    const Ciphertext &Matrix::operator()(bool colwise, size_t idx, bool) const { return elems[idx_to_idx(colwise, idx)]; }
    Ciphertext &Matrix::operator()(bool colwise, size_t idx, bool) { return elems[idx_to_idx(colwise, idx)]; }
    const Ciphertext &Matrix::operator()(size_t i, size_t j) const { return elems[ij_to_idx(i, j)]; }
    Ciphertext &Matrix::operator()(size_t i, size_t j) { return elems[ij_to_idx(i, j)]; }
    void Matrix::set_elem(size_t i, size_t j, const Ciphertext &e) { elems[ij_to_idx(i, j)] = e; }
    void Matrix::set_elem(size_t i, size_t j, Ciphertext &&e) { elems[ij_to_idx(i, j)] = std::move(e); }

    // column-major storage; a transposed view swaps the roles of i and j (he_linalg.cpp:376-384)
    size_t Matrix::ij_to_idx(size_t i, size_t j) const
    {
        return (transposed ? j : i) + dims[0] * (transposed ? i : j);
    }
    size_t Matrix::idx_to_idx(bool colwise, size_t idx) const
    {
        return transposed != colwise ? idx : idx / dims[1] + idx % dims[1] * dims[0];
    }

    Matrix &Matrix::operator-=(const Evaluator &eval)
    {
        for (size_t idx = 0; idx < dims[0] * dims[1]; ++idx) elems[idx] -= eval;
        return *this;
    }
    Matrix operator-(const tuple<const Evaluator &, const Matrix &> &e)
    {
        Matrix r = get<1>(e);
        return r -= get<0>(e);
    }
    Matrix &Matrix::operator+=(const tuple<const Evaluator &, const Matrix &> &e)
    {
        const Evaluator &eval = get<0>(e);
        const Matrix &o = get<1>(e);
        const vector<size_t> d = get_dims();
        assert(d == o.get_dims());
        for (size_t j = 0; j < d[1]; ++j)
            for (size_t i = 0; i < d[0]; ++i) (*this)(i, j) += eval % o(i, j);
        return *this;
    }
    Matrix operator+(const tuple<const Evaluator &, const Matrix &> &e, const Matrix &b)
    {
        Matrix r = get<1>(e);
        return r += get<0>(e) % b;
    }
    Matrix &Matrix::operator-=(const tuple<const Evaluator &, const Matrix &> &e)
    {
        const Evaluator &eval = get<0>(e);
        const Matrix &o = get<1>(e);
        const vector<size_t> d = get_dims();
        assert(d == o.get_dims());
        for (size_t j = 0; j < d[1]; ++j)
            for (size_t i = 0; i < d[0]; ++i) (*this)(i, j) -= eval % o(i, j);
        return *this;
    }
    Matrix operator-(const tuple<const Evaluator &, const Matrix &> &e, const Matrix &b)
    {
        Matrix r = get<1>(e);
        return r -= get<0>(e) % b;
    }
    Matrix &Matrix::operator*=(const tuple<const EvalRk &, const Matrix &> &e)
    {
        const Evaluator &eval = get<0>(get<0>(e));
        const RelinKeys &rk = get<1>(get<0>(e));
        const Matrix &o = get<1>(e);
        const vector<size_t> d = get_dims();
        assert(d == o.get_dims());
        for (size_t j = 0; j < d[1]; ++j)
            for (size_t i = 0; i < d[0]; ++i) {
                Ciphertext &x = (*this)(i, j);
                x *= eval % o(i, j);
                x &= eval % rk;  // relin
                x ^= eval;       // rescale
            }
        return *this;
    }
    Matrix operator*(const tuple<const EvalRk &, const Matrix &> &e, const Matrix &b)
    {
        Matrix r = get<1>(e);
        return r *= get<0>(e) % b;
    }

    // res(i, j) = relin+rescale( sum_k A(i, k) * B(k, j) ) for the views (a, a_tr), (b, b_tr)
    Matrix Matrix::product(const Evaluator &eval, const RelinKeys &rk, const Matrix &a, bool a_tr, const Matrix &b,
                           bool b_tr)
    {
        const size_t r1 = a_tr ? a.dims[1] : a.dims[0], c1 = a_tr ? a.dims[0] : a.dims[1];
        const size_t r2 = b_tr ? b.dims[1] : b.dims[0], c2 = b_tr ? b.dims[0] : b.dims[1];
        assert(c1 == r2);
        (void)c1;
        (void)r2;
        vector<const hec_ciphertext *> pa, pb;
        for (const auto &x : a.elems) pa.push_back(x.get());
        for (const auto &x : b.elems) pb.push_back(x.get());
        vector<Ciphertext> out;
        vector<hec_ciphertext *> po;
        out.reserve(r1 * c2);
        for (size_t k = 0; k < r1 * c2; ++k) {
            out.emplace_back(eval.context());
            po.push_back(out.back().get());
        }
        hecdna::check(hec_matrix_matmul(eval.context().get(), pa.data(), a.dims[0], a.dims[1], a_tr ? 1 : 0, pb.data(),
                                        b.dims[0], b.dims[1], b_tr ? 1 : 0, rk.get(), po.data()));
        return Matrix(r1, c2, std::move(out));
    }

    Matrix Matrix::matmul(const Evaluator &eval, const RelinKeys &rk, const Matrix &other) const
    {
        assert(get_dims()[1] == other.get_dims()[0]);
        return product(eval, rk, *this, transposed, other, other.transposed);
    }
    Matrix Matrix::left_matmul_with_transp(const Evaluator &eval, const RelinKeys &rk) const
    {
        return product(eval, rk, *this, !transposed, *this, transposed);  // this^T * this
    }
    Matrix Matrix::matmul_square(const Evaluator &eval, const RelinKeys &rk) const
    {
        assert(dims[0] == dims[1]);
        return product(eval, rk, *this, transposed, *this, transposed);
    }
    // square-and-multiply over matmul_square / matmul (he_linalg.cpp:316-349)
    Matrix Matrix::matmul_pow(const Evaluator &eval, const RelinKeys &rk, int powr) const
    {
        assert(dims[0] == dims[1]);
        Matrix res(dims[0], dims[0]);
        Matrix acc = *this;
        const int nbits = (int)std::ceil(std::log2(powr + 1));
        bool have = false;
        if (powr & 1) {
            res = acc;
            have = true;
        }
        for (int i = 1; i < nbits; ++i) {
            acc = acc.matmul_square(eval, rk);
            if ((powr >> i) & 1) {
                if (!have) {
                    res = acc;
                    have = true;
                } else {
                    res = res.matmul(eval, rk, acc);
                }
            }
        }
        return res;
    }

    // =================================================================== BatchedVector
    BatchedVector::BatchedVector(size_t d, const Ciphertext &c) : dim(d), bvec(c) {}
    BatchedVector::BatchedVector(size_t d, Ciphertext &&c) : dim(d), bvec(std::move(c)) {}
    size_t BatchedVector::get_dim() const { return dim; }
    const Ciphertext &BatchedVector::get_bvec() const { return bvec; }

    BatchedVector &BatchedVector::operator-=(const Evaluator &eval) { bvec -= eval; return *this; }
    BatchedVector operator-(const tuple<const Evaluator &, const BatchedVector &> &e)
    {
        BatchedVector r = get<1>(e);
        return r -= get<0>(e);
    }
    BatchedVector &BatchedVector::operator+=(const tuple<const Evaluator &, const BatchedVector &> &e)
    {
        bvec += get<0>(e) % get<1>(e).bvec;
        return *this;
    }
    BatchedVector operator+(const tuple<const Evaluator &, const BatchedVector &> &e, const BatchedVector &b)
    {
        BatchedVector r = get<1>(e);
        return r += get<0>(e) % b;
    }
    BatchedVector &BatchedVector::operator-=(const tuple<const Evaluator &, const BatchedVector &> &e)
    {
        bvec -= get<0>(e) % get<1>(e).bvec;
        return *this;
    }
    BatchedVector operator-(const tuple<const Evaluator &, const BatchedVector &> &e, const BatchedVector &b)
    {
        BatchedVector r = get<1>(e);
        return r -= get<0>(e) % b;
    }
    BatchedVector &BatchedVector::operator*=(const tuple<const Evaluator &, const BatchedVector &> &e)
    {
        bvec *= get<0>(e) % get<1>(e).bvec;
        return *this;
    }
    BatchedVector operator*(const tuple<const Evaluator &, const BatchedVector &> &e, const BatchedVector &b)
    {
        BatchedVector r = get<1>(e);
        return r *= get<0>(e) % b;
    }
    BatchedVector &BatchedVector::operator&=(const EvalRk &e)
    {
        bvec &= get<0>(e) % get<1>(e);
        return *this;
    }
    BatchedVector operator&(const EvalRk &e, const BatchedVector &a)
    {
        BatchedVector r = a;
        return r &= e;
    }
    BatchedVector &BatchedVector::operator^=(const Evaluator &eval) { bvec ^= eval; return *this; }
    BatchedVector operator^(const Evaluator &eval, const BatchedVector &a)
    {
        BatchedVector r = a;
        return r ^= eval;
    }
    BatchedVector &BatchedVector::operator*=(const tuple<const EvalRk &, const BatchedVector &> &e)
    {
        const Evaluator &eval = get<0>(get<0>(e));
        *this *= eval % get<1>(e);
        *this &= get<0>(e);  // relin
        *this ^= eval;       // rescale
        return *this;
    }
    BatchedVector operator*(const tuple<const EvalRk &, const BatchedVector &> &e, const BatchedVector &b)
    {
        BatchedVector r = get<1>(e);
        return r *= get<0>(e) % b;
    }
    BatchedVector &BatchedVector::operator<<=(const tuple<const EvalGk &, const int &> &e)
    {
        get<0>(get<0>(e)).rotate_vector_inplace(bvec, get<1>(e), get<1>(get<0>(e)));
        return *this;
    }
    BatchedVector operator<<(const tuple<const EvalGk &, const BatchedVector &> &e, int steps)
    {
        BatchedVector r = get<1>(e);
        get<0>(get<0>(e)).rotate_vector(get<1>(e).bvec, steps, get<1>(get<0>(e)), r.bvec);
        return r;
    }
    BatchedVector &BatchedVector::operator>>=(const tuple<const EvalGk &, const int &> &e)
    {
        get<0>(get<0>(e)).rotate_vector_inplace(bvec, -get<1>(e), get<1>(get<0>(e)));
        return *this;
    }
    BatchedVector operator>>(const tuple<const EvalGk &, const BatchedVector &> &e, int steps)
    {
        BatchedVector r = get<1>(e);
        get<0>(get<0>(e)).rotate_vector(get<1>(e).bvec, -steps, get<1>(get<0>(e)), r.bvec);
        return r;
    }
    BatchedVector &BatchedVector::square_inplace(const Evaluator &eval, const RelinKeys &rk)
    {
        eval.square_inplace(bvec);
        bvec &= eval % rk;  // relin
        bvec ^= eval;       // rescale
        return *this;
    }
    BatchedVector BatchedVector::square(const Evaluator &eval, const RelinKeys &rk) const
    {
        BatchedVector r = *this;
        r.square_inplace(eval, rk);
        return r;
    }
    // log-step rotate-and-add over the binary expansion of dim (he_linalg.cpp:667-713)
    BatchedVector &BatchedVector::sum_elems_inplace(const Evaluator &eval, const GaloisKeys &gk)
    {
        using he::operators::operator+;
        using he::operators::operator<<;
        const auto egk = eval % gk;
        Ciphertext to_sum = bvec, partial, tmp;
        int window = 1;
        bool have = false;
        if (dim & 1) {
            have = true;
            to_sum <<= egk % window;
        }
        for (size_t bits = dim >> 1; bits != 0; bits >>= 1) {
            window <<= 1;
            if (bits & 1) {
                int steps = window >> 1;
                tmp = egk % to_sum << steps;
                Ciphertext &acc = have ? partial : bvec;
                acc = eval % to_sum + tmp;
                for (steps >>= 1; steps != 0; steps >>= 1) {
                    tmp = egk % acc << steps;
                    acc += eval % tmp;
                }
                if (have) bvec += eval % partial;
                else have = true;
                if (bits != 1) to_sum <<= egk % window;
            }
        }
        dim = 1;
        return *this;
    }
    BatchedVector BatchedVector::sum_elems(const Evaluator &eval, const GaloisKeys &gk)
    {
        BatchedVector r = *this;
        r.sum_elems_inplace(eval, gk);
        return r;
    }

    // =================================================================== BatchedMatrix
    BatchedMatrix::BatchedMatrix(BatchingType t, const vector<BatchedVector> &v) : btype(t), bvecs(v) {}
    BatchedMatrix::BatchedMatrix(BatchingType t, vector<BatchedVector> &&v) : btype(t), bvecs(std::move(v)) {}
    BatchedMatrix::BatchingType BatchedMatrix::get_btype() const { return btype; }
    bool BatchedMatrix::get_transp() const { return transposed; }
    void BatchedMatrix::transp() { transposed = !transposed; }
    size_t BatchedMatrix::get_col_dim() const { return !transposed ? bvecs.size() : bvecs[0].get_dim(); }
    size_t BatchedMatrix::get_row_dim() const { return transposed ? bvecs.size() : bvecs[0].get_dim(); }
    const vector<BatchedVector> &BatchedMatrix::get_bvecs() const { return bvecs; }
    const BatchedVector &BatchedMatrix::operator[](size_t i) const { return bvecs[i]; }
    BatchedVector &BatchedMatrix::operator[](size_t i) { return bvecs[i]; }

    BatchedMatrix &BatchedMatrix::operator-=(const Evaluator &eval)
    {
        for (auto &b : bvecs) b -= eval;
        return *this;
    }
    BatchedMatrix operator-(const tuple<const Evaluator &, const BatchedMatrix &> &e)
    {
        BatchedMatrix r = get<1>(e);
        return r -= get<0>(e);
    }
    BatchedMatrix &BatchedMatrix::operator+=(const tuple<const Evaluator &, const BatchedMatrix &> &e)
    {
        const BatchedMatrix &o = get<1>(e);
        assert(transposed == o.transposed);
        for (size_t i = 0; i < bvecs.size(); ++i) bvecs[i] += get<0>(e) % o.bvecs[i];
        return *this;
    }
    BatchedMatrix operator+(const tuple<const Evaluator &, const BatchedMatrix &> &e, const BatchedMatrix &b)
    {
        BatchedMatrix r = get<1>(e);
        return r += get<0>(e) % b;
    }
    BatchedMatrix &BatchedMatrix::operator-=(const tuple<const Evaluator &, const BatchedMatrix &> &e)
    {
        const BatchedMatrix &o = get<1>(e);
        assert(transposed == o.transposed);
        for (size_t i = 0; i < bvecs.size(); ++i) bvecs[i] -= get<0>(e) % o.bvecs[i];
        return *this;
    }
    BatchedMatrix operator-(const tuple<const Evaluator &, const BatchedMatrix &> &e, const BatchedMatrix &b)
    {
        BatchedMatrix r = get<1>(e);
        return r -= get<0>(e) % b;
    }
    BatchedMatrix &BatchedMatrix::operator*=(const tuple<const EvalRk &, const BatchedMatrix &> &e)
    {
        const BatchedMatrix &o = get<1>(e);
        assert(transposed == o.transposed);
        for (size_t i = 0; i < bvecs.size(); ++i) bvecs[i] *= get<0>(e) % o.bvecs[i];
        return *this;
    }
    BatchedMatrix operator*(const tuple<const EvalRk &, const BatchedMatrix &> &e, const BatchedMatrix &b)
    {
        BatchedMatrix r = get<1>(e);
        return r *= get<0>(e) % b;
    }
    BatchedMatrix &BatchedMatrix::square_inplace(const Evaluator &eval, const RelinKeys &rk)
    {
        for (auto &b : bvecs) b.square_inplace(eval, rk);
        return *this;
    }
    BatchedMatrix BatchedMatrix::square(const Evaluator &eval, const RelinKeys &rk) const
    {
        BatchedMatrix r = *this;
        r.square_inplace(eval, rk);
        return r;
    }
    BatchedMatrix &BatchedMatrix::sum_bvec_elems_inplace(const Evaluator &eval, const GaloisKeys &gk)
    {
        for (auto &b : bvecs) b.sum_elems_inplace(eval, gk);
        return *this;
    }
    BatchedMatrix BatchedMatrix::sum_bvec_elems(const Evaluator &eval, const GaloisKeys &gk)
    {
        BatchedMatrix r = *this;
        r.sum_bvec_elems_inplace(eval, gk);
        return r;
    }

    // he_linalg.cpp:943-1006 — one batched engine call for all p output vectors
    BatchedMatrix BatchedMatrix::matmul(const Evaluator &eval, const RelinKeys &rk, const GaloisKeys &gk,
                                        const BatchedMatrix &other) const
    {
        assert(other.btype == BatchingType::col);
        assert(!transposed);
        const size_t n = get_col_dim(), p = other.get_col_dim();
        const bool col = btype == BatchingType::col;
        vector<const hec_ciphertext *> pa, pb;
        for (const auto &b : bvecs) pa.push_back(b.bvec.get());
        for (const auto &b : other.bvecs) pb.push_back(b.bvec.get());
        vector<Ciphertext> out;
        vector<hec_ciphertext *> po;
        out.reserve(p);
        for (size_t i = 0; i < p; ++i) {
            out.emplace_back(eval.context());
            po.push_back(out.back().get());
        }
        if (col) {  // col x col^T -> diag batched result
            assert(other.transposed);
            assert(n == other.get_row_dim());
            hecdna::check(hec_matmul_col_colT(eval.context().get(), pa.data(), n, pb.data(), p, rk.get(), gk.get(),
                                              po.data()));
        } else {    // diag x col -> col batched result (the matvec)
            assert(!other.transposed);
            if (eval.context().has_comm())  // sharded over the ranks of the context's communicator
                hecdna::check(hec_matmul_diag_col_sharded(eval.context().get(), pa.data(), n, pb.data(), p, rk.get(),
                                                          gk.get(), po.data()));
            else
                hecdna::check(hec_matmul_diag_col(eval.context().get(), pa.data(), n, pb.data(), p, rk.get(),
                                                  gk.get(), po.data()));
        }
        vector<BatchedVector> res;
        res.reserve(p);
        for (size_t i = 0; i < p; ++i) res.emplace_back(other.bvecs[col ? 0 : i].dim, std::move(out[i]));
        return BatchedMatrix(col ? BatchingType::diag : BatchingType::col, std::move(res));
    }
} // namespace he::linalg
