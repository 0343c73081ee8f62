#pragma once
// Drop-in for the reference's he::linalg (include/he_linalg.h:7-413) over hecdna types: same
// classes, constructors, operators and member functions.  The hot paths BatchedMatrix::matmul
// (he_linalg.cpp:943-1006) and Matrix::matmul (:202-236) run as one batched engine call each
// (hec_matmul_diag_col / hec_matmul_col_colT / hec_matrix_matmul) with bit-identical results.
#include <concepts>
#include <cstddef>
#include <tuple>
#include <vector>

#include "he_operators.h"

namespace he::linalg
{
    class Matrix;
    class BatchedVector;
    class BatchedMatrix;

    template <typename T>
    concept Matrix_BatchedVector_BatchedMatrix_tn = std::same_as<std::decay_t<T>, Matrix> ||
                                                    std::same_as<std::decay_t<T>, BatchedVector> ||
                                                    std::same_as<std::decay_t<T>, BatchedMatrix>;

    template <Matrix_BatchedVector_BatchedMatrix_tn T>
    constexpr auto operator%(const hecdna::Evaluator &eval, T &&op)
    {
        return std::tie(eval, std::forward<T>(op));
    }
    template <Matrix_BatchedVector_BatchedMatrix_tn T>
    constexpr auto operator%(const std::tuple<const hecdna::Evaluator &, const hecdna::RelinKeys &> &eval_rk, T &&op)
    {
        return std::tie(eval_rk, std::forward<T>(op));
    }
    template <Matrix_BatchedVector_BatchedMatrix_tn T>
    constexpr auto operator%(const std::tuple<const hecdna::Evaluator &, const hecdna::GaloisKeys &> &eval_gk, T &&op)
    {
        return std::tie(eval_gk, std::forward<T>(op));
    }

    using EvalRk = std::tuple<const hecdna::Evaluator &, const hecdna::RelinKeys &>;
    using EvalGk = std::tuple<const hecdna::Evaluator &, const hecdna::GaloisKeys &>;

    // -----------------------------------
    class Matrix
    {
    public:
        Matrix() = delete;
        Matrix(const Matrix &copy) = default;
        Matrix(Matrix &&source) = default;
        ~Matrix() = default;
        Matrix &operator=(const Matrix &copy) = default;
        Matrix &operator=(Matrix &&source) = default;

        Matrix(std::size_t rows, std::size_t cols, const std::vector<hecdna::Ciphertext> &elems);
        Matrix(std::size_t rows, std::size_t cols, std::vector<hecdna::Ciphertext> &&elems);
        Matrix(std::size_t rows, std::size_t cols);

        std::vector<std::size_t> get_dims() const;
        void transp();
        bool get_transp() const;
        const std::vector<hecdna::Ciphertext> &get_elems() const;
        const hecdna::Ciphertext &operator()(bool colwise, std::size_t idx, bool dummy_arg) const;
        hecdna::Ciphertext &operator()(bool colwise, std::size_t idx, bool dummy_arg);
        const hecdna::Ciphertext &operator()(std::size_t i, std::size_t j) const;
        hecdna::Ciphertext &operator()(std::size_t i, std::size_t j);
        void set_elem(std::size_t i, std::size_t j, const hecdna::Ciphertext &elem);
        void set_elem(std::size_t i, std::size_t j, hecdna::Ciphertext &&elem);

        Matrix &operator-=(const hecdna::Evaluator &eval);
        friend Matrix operator-(const std::tuple<const hecdna::Evaluator &, const Matrix &> &eval_op);
        Matrix &operator+=(const std::tuple<const hecdna::Evaluator &, const Matrix &> &eval_other);
        friend Matrix operator+(const std::tuple<const hecdna::Evaluator &, const Matrix &> &eval_op1, const Matrix &op2);
        Matrix &operator-=(const std::tuple<const hecdna::Evaluator &, const Matrix &> &eval_other);
        friend Matrix operator-(const std::tuple<const hecdna::Evaluator &, const Matrix &> &eval_op1, const Matrix &op2);
        Matrix &operator*=(const std::tuple<const EvalRk &, const Matrix &> &eval_rk__other);
        friend Matrix operator*(const std::tuple<const EvalRk &, const Matrix &> &eval_rk__op1, const Matrix &op2);

        Matrix matmul(const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk, const Matrix &other) const;
        Matrix left_matmul_with_transp(const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk) const;
        Matrix matmul_square(const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk) const;
        Matrix matmul_pow(const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk, int powr) const;

    private:
        std::size_t ij_to_idx(std::size_t i, std::size_t j) const;
        std::size_t idx_to_idx(bool colwise, std::size_t idx) const;
        static Matrix product(const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk, const Matrix &a, bool a_tr,
                              const Matrix &b, bool b_tr);

        std::vector<std::size_t> dims;
        bool transposed = false;
        std::vector<hecdna::Ciphertext> elems{};
    };

    // -----------------------------------
    class BatchedVector
    {
    public:
        BatchedVector() = delete;
        BatchedVector(const BatchedVector &copy) = default;
        BatchedVector(BatchedVector &&source) = default;
        ~BatchedVector() = default;
        BatchedVector &operator=(const BatchedVector &copy) = default;
        BatchedVector &operator=(BatchedVector &&source) = default;

        BatchedVector(std::size_t dim, const hecdna::Ciphertext &bvec);
        BatchedVector(std::size_t dim, hecdna::Ciphertext &&bvec);

        std::size_t get_dim() const;
        const hecdna::Ciphertext &get_bvec() const;

        BatchedVector &operator-=(const hecdna::Evaluator &eval);
        friend BatchedVector operator-(const std::tuple<const hecdna::Evaluator &, const BatchedVector &> &eval_op);
        BatchedVector &operator+=(const std::tuple<const hecdna::Evaluator &, const BatchedVector &> &eval_other);
        friend BatchedVector operator+(const std::tuple<const hecdna::Evaluator &, const BatchedVector &> &eval_op1,
                                       const BatchedVector &op2);
        BatchedVector &operator-=(const std::tuple<const hecdna::Evaluator &, const BatchedVector &> &eval_other);
        friend BatchedVector operator-(const std::tuple<const hecdna::Evaluator &, const BatchedVector &> &eval_op1,
                                       const BatchedVector &op2);
        BatchedVector &operator*=(const std::tuple<const hecdna::Evaluator &, const BatchedVector &> &eval_other);
        friend BatchedVector operator*(const std::tuple<const hecdna::Evaluator &, const BatchedVector &> &eval_op1,
                                       const BatchedVector &op2);
        BatchedVector &operator&=(const EvalRk &eval_rk);
        friend BatchedVector operator&(const EvalRk &eval_rk, const BatchedVector &op);
        BatchedVector &operator^=(const hecdna::Evaluator &eval);
        friend BatchedVector operator^(const hecdna::Evaluator &eval, const BatchedVector &op);
        BatchedVector &operator*=(const std::tuple<const EvalRk &, const BatchedVector &> &eval_rk__other);
        friend BatchedVector operator*(const std::tuple<const EvalRk &, const BatchedVector &> &eval_rk__op1,
                                       const BatchedVector &op2);
        BatchedVector &operator<<=(const std::tuple<const EvalGk &, const int &> &eval_gk__steps);
        friend BatchedVector operator<<(const std::tuple<const EvalGk &, const BatchedVector &> &eval_gk__op, int steps);
        BatchedVector &operator>>=(const std::tuple<const EvalGk &, const int &> &eval_gk__steps);
        friend BatchedVector operator>>(const std::tuple<const EvalGk &, const BatchedVector &> &eval_gk__op, int steps);

        BatchedVector &square_inplace(const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk);
        BatchedVector square(const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk) const;
        BatchedVector &sum_elems_inplace(const hecdna::Evaluator &eval, const hecdna::GaloisKeys &gk);
        BatchedVector sum_elems(const hecdna::Evaluator &eval, const hecdna::GaloisKeys &gk);

    private:
        friend class BatchedMatrix;
        std::size_t dim;
        hecdna::Ciphertext bvec;
    };

    // -----------------------------------
    class BatchedMatrix
    {
    public:
        BatchedMatrix() = delete;
        BatchedMatrix(const BatchedMatrix &copy) = default;
        BatchedMatrix(BatchedMatrix &&source) = default;
        ~BatchedMatrix() = default;
        BatchedMatrix &operator=(const BatchedMatrix &copy) = default;
        BatchedMatrix &operator=(BatchedMatrix &&source) = default;

        enum class BatchingType { col, diag };

        BatchedMatrix(BatchingType btype, const std::vector<BatchedVector> &bvecs);
        BatchedMatrix(BatchingType btype, std::vector<BatchedVector> &&bvecs);

        BatchingType get_btype() const;
        std::size_t get_col_dim() const;
        std::size_t get_row_dim() const;
        bool get_transp() const;
        void transp();
        const std::vector<BatchedVector> &get_bvecs() const;
        const BatchedVector &operator[](std::size_t i) const;
        BatchedVector &operator[](std::size_t i);

        BatchedMatrix &operator-=(const hecdna::Evaluator &eval);
        friend BatchedMatrix operator-(const std::tuple<const hecdna::Evaluator &, const BatchedMatrix &> &eval_op);
        BatchedMatrix &operator+=(const std::tuple<const hecdna::Evaluator &, const BatchedMatrix &> &eval_other);
        friend BatchedMatrix operator+(const std::tuple<const hecdna::Evaluator &, const BatchedMatrix &> &eval_op1,
                                       const BatchedMatrix &op2);
        BatchedMatrix &operator-=(const std::tuple<const hecdna::Evaluator &, const BatchedMatrix &> &eval_other);
        friend BatchedMatrix operator-(const std::tuple<const hecdna::Evaluator &, const BatchedMatrix &> &eval_op1,
                                       const BatchedMatrix &op2);
        BatchedMatrix &operator*=(const std::tuple<const EvalRk &, const BatchedMatrix &> &eval_rk__other);
        friend BatchedMatrix operator*(const std::tuple<const EvalRk &, const BatchedMatrix &> &eval_rk__op1,
                                       const BatchedMatrix &op2);
        BatchedMatrix &square_inplace(const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk);
        BatchedMatrix square(const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk) const;
        BatchedMatrix &sum_bvec_elems_inplace(const hecdna::Evaluator &eval, const hecdna::GaloisKeys &gk);
        BatchedMatrix sum_bvec_elems(const hecdna::Evaluator &eval, const hecdna::GaloisKeys &gk);

        BatchedMatrix matmul(const hecdna::Evaluator &eval, const hecdna::RelinKeys &rk, const hecdna::GaloisKeys &gk,
                             const BatchedMatrix &other) const;

    private:
        BatchingType btype;
        bool transposed = false;
        std::vector<BatchedVector> bvecs;
    };
} // namespace he::linalg
