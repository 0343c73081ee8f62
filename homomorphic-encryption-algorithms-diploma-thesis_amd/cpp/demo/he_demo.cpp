// he_demo — the reference's `demo matrix_operations batched_matmul_ckks` flow
// (src/demos/matrix_operations.cpp:1042-1175) written against the hecdna drop-in headers:
// identical he::operators / he::linalg code, with seal:: types replaced by hecdna:: types.
// Key generation / encryption / decryption stay with the caller (SEAL in a real deployment); this
// program reads SEAL-layout keys and ciphertexts from a file and writes the result ciphertexts.
//
// usage: he_demo <mode> <in.bin> <out.bin>
//   mode = batched_diag   (COL_OR_DIAG = 1: A diag-batched x B col-batched)
//          batched_col    (COL_OR_DIAG = 0: A col-batched x A^T)
//          ops            (operator expressions: ((eval%gk%c0) << 5) * c1, relin, rescale, + c2 ...)
//          matrix         (Matrix 2x2 elementwise-ciphertext matmul, he_linalg.cpp:202-236)
//          matrix_family  (left_matmul_with_transp, matmul_square, matmul_pow, he_linalg.cpp:241-349)
//          server         (server.cpp:99-152 on SEAL-serialized parms, relin key and two ciphertexts; the
//                          result written with Ciphertext::save)
//          encode         (the demo's plaintexts: CKKSEncoder::encode of mat1's columns, the data of
//                          matrix_operations.cpp:1079-1087 at dim = #ciphertexts in the input, scale 2^40,
//                          matrix_operations.cpp:1106-1108; written as size-1 entries)
//          math:<iter>    (he::math on the he_math.h drop-in: signed_inv(c0, 1.0), inv_sqrt_twice(c0, 0.7),
//                          sqrt(c0, 1.0), abs(c1, 1.0) with <iter> iterations, src/core/he_math.cpp:22-269)
//          util           (he::util: drop_chain_levels(c0, 2), then reach_chain_level of {c1, c2} to c0's level,
//                          include/he_util.h:27-77; the chain indices of every output are printed)
//          least_squares  (src/demos/matrix_operations.cpp:915-1003 on x = c0, y = c1 of 5 data slots: the sums,
//                          the denominator, signed_inv(denom, 0.05, 6), the numerators, a and b)
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <map>
#include <string>
#include <vector>

#include "he_linalg.h"
#include "he_math.h"
#include "he_operators.h"
#include "he_util.h"

using namespace he::operators;
using namespace he::linalg;
using hecdna::Ciphertext;

namespace {
struct Input {
    std::uint64_t N = 0;
    std::vector<std::uint64_t> moduli;
    struct Ct { std::uint64_t size, level; double scale; std::vector<std::uint64_t> data; };
    std::vector<Ct> cts;
    std::vector<std::uint64_t> rk;
    std::map<std::uint32_t, std::vector<std::uint64_t>> gk;
};

template <class T>
void rd(std::ifstream &f, T *p, std::size_t n)
{
    f.read(reinterpret_cast<char *>(p), sizeof(T) * n);
    if (!f) throw std::runtime_error("truncated input");
}

Input read_input(const char *path)
{
    std::ifstream f(path, std::ios::binary);
    char magic[8];
    rd(f, magic, 8);
    if (std::memcmp(magic, "HECDNA01", 8)) throw std::runtime_error("bad magic");
    Input in;
    std::uint64_t K, n;
    rd(f, &in.N, 1);
    rd(f, &K, 1);
    in.moduli.resize(K);
    rd(f, in.moduli.data(), K);
    rd(f, &n, 1);
    for (std::uint64_t i = 0; i < n; ++i) {
        Input::Ct c;
        rd(f, &c.size, 1);
        rd(f, &c.level, 1);
        rd(f, &c.scale, 1);
        c.data.resize(c.size * c.level * in.N);
        rd(f, c.data.data(), c.data.size());
        in.cts.push_back(std::move(c));
    }
    const std::size_t kw = (K - 1) * 2 * K * in.N;
    std::uint64_t has_rk, ngk;
    rd(f, &has_rk, 1);
    if (has_rk) {
        in.rk.resize(kw);
        rd(f, in.rk.data(), kw);
    }
    rd(f, &ngk, 1);
    for (std::uint64_t i = 0; i < ngk; ++i) {
        std::uint64_t elt;
        rd(f, &elt, 1);
        auto &v = in.gk[(std::uint32_t)elt];
        v.resize(kw);
        rd(f, v.data(), kw);
    }
    return in;
}

void write_output(const char *path, const std::vector<const Ciphertext *> &cts)
{
    std::ofstream f(path, std::ios::binary);
    const std::uint64_t n = cts.size();
    f.write(reinterpret_cast<const char *>(&n), 8);
    for (const Ciphertext *c : cts) {
        const std::uint64_t s = c->size(), l = c->level();
        const double sc = c->scale();
        const auto d = c->download();
        f.write(reinterpret_cast<const char *>(&s), 8);
        f.write(reinterpret_cast<const char *>(&l), 8);
        f.write(reinterpret_cast<const char *>(&sc), 8);
        f.write(reinterpret_cast<const char *>(d.data()), d.size() * 8);
    }
}
}  // namespace

int main(int argc, char **argv)
{
    if (argc != 4) {
        std::cout << "usage: he_demo <batched_diag|batched_col|ops|matrix|matrix_family|encode|sum_elems:<dim>|math:<iter>|"
                     "util|least_squares|server> <in.bin> <out.bin>\n";
        return 1;
    }
    const std::string mode = argv[1];
    if (mode == "server") {
        // src/demos/server.cpp:99-152 (server_demo's receive / compute / send) over the SEAL wire format: the input
        // file is the client's network buffer (EncryptionParameters, RelinKeys, two Ciphertexts, as client.cpp
        // writes them); the output file is res_ct.save(onet_strm), SEAL's default zstd compression
        std::ifstream f(argv[2], std::ios::binary);
        std::vector<char> raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        const auto *inet_buf = reinterpret_cast<const hecdna::seal_byte *>(raw.data());
        const std::streamoff inet_buf_sz = (std::streamoff)raw.size();
        hecdna::EncryptionParameters parms;
        std::streamoff inet_buf_curpos = 0;
        inet_buf_curpos += parms.load(inet_buf + inet_buf_curpos, inet_buf_sz - inet_buf_curpos);
        hecdna::Context sctx(parms);
        hecdna::RelinKeys srk;
        inet_buf_curpos += srk.load(sctx, inet_buf + inet_buf_curpos, inet_buf_sz - inet_buf_curpos);
        Ciphertext op1_ct, op2_ct;
        inet_buf_curpos += op1_ct.load(sctx, inet_buf + inet_buf_curpos, inet_buf_sz - inet_buf_curpos);
        inet_buf_curpos += op2_ct.load(sctx, inet_buf + inet_buf_curpos, inet_buf_sz - inet_buf_curpos);
        hecdna::Evaluator seval(sctx);
        Ciphertext res_ct;
        res_ct = seval % op1_ct * op2_ct;
        res_ct &= seval % srk;  // relin
        res_ct ^= seval;        // rescale
        std::ofstream onet_strm(argv[3], std::ios::binary);
        const std::streamoff n = res_ct.save(onet_strm);
        std::cout << "he_demo server: read " << inet_buf_curpos << " bytes, wrote " << n << " bytes\n";
        return 0;
    }
    const Input in = read_input(argv[2]);

    hecdna::Context ctx(in.N, in.moduli);  // SEALContext ctx(parms)
    hecdna::Evaluator eval(ctx);           // Evaluator eval(ctx)
    hecdna::RelinKeys rk;
    if (!in.rk.empty()) rk = hecdna::RelinKeys(ctx, in.rk.data());
    hecdna::GaloisKeys gk(ctx);
    for (const auto &[elt, data] : in.gk) gk.add(elt, data.data());
    std::vector<Ciphertext> cts;
    for (const auto &c : in.cts) {
        cts.emplace_back(ctx);
        cts.back().upload(c.data.data(), c.size, c.level, c.scale);
    }

    std::vector<const Ciphertext *> outs;
    std::vector<Ciphertext> keep;
    if (mode == "batched_diag_sharded")  // the same demo with the context on a (one-rank) RCCL communicator
        ctx.comm_init(0, 1, hecdna::Context::comm_unique_id());
    if (mode == "batched_diag_sharded_host") {  // ... on a host communicator (hec_comm_init_ops) of a one-rank world:
        // the all-reduces over one rank are the identity, so the partials still take the host exchange path
        // (download, allreduce_u64_sum, upload) and the agreement step
        hec_comm_ops ops{};
        ops.allreduce_f64 = [](void *, double *, uint64_t, int) { return 0; };
        ops.allreduce_u64_sum = [](void *, uint64_t *, uint64_t) { return 0; };
        ctx.comm_init(0, 1, ops);
    }
    if (mode == "batched_diag" || mode == "batched_col" || mode == "batched_diag_sharded" ||
        mode == "batched_diag_sharded_host") {
        // matrix_operations.cpp:1112-1141 — the same code the reference runs over seal:: types
        const std::size_t dim = cts.size();
        std::vector<BatchedVector> mat1_cols_bvec;
        mat1_cols_bvec.reserve(dim);
        for (std::size_t i = 0; i < dim; ++i) mat1_cols_bvec.emplace_back(dim, cts[i]);
        std::vector<BatchedVector> res;
        if (mode != "batched_col") {
            BatchedMatrix mat1_bmat(BatchedMatrix::BatchingType::diag, mat1_cols_bvec);
            BatchedMatrix mat2_bmat(BatchedMatrix::BatchingType::col, std::move(mat1_cols_bvec));
            BatchedMatrix mat3_bmat = mat1_bmat.matmul(eval, rk, gk, mat2_bmat);
            res = mat3_bmat.get_bvecs();
        } else {
            BatchedMatrix mat1_bmat(BatchedMatrix::BatchingType::col, std::move(mat1_cols_bvec));
            BatchedMatrix mat2_bmat = mat1_bmat;
            mat2_bmat.transp();
            BatchedMatrix mat3_bmat = mat1_bmat.matmul(eval, rk, gk, mat2_bmat);
            res = mat3_bmat.get_bvecs();
        }
        for (auto &b : res) keep.push_back(b.get_bvec());
    } else if (mode == "ops") {
        // operator surface of he_operators.h on three ciphertexts
        Ciphertext r = eval % gk % cts[0] << 5;  // rotate left
        r *= eval % cts[1];                       // ct x ct
        r &= eval % rk;                           // relinearize
        r ^= eval;                                // rescale
        Ciphertext s = eval % gk % cts[2] >> 3;   // rotate right (out of place)
        s |= eval;                                // mod switch to next
        keep.push_back(r);
        keep.push_back(s);
        Ciphertext t = eval % cts[0] - cts[1];
        t -= eval;                                // negate
        keep.push_back(t);
    } else if (mode.rfind("sum_elems:", 0) == 0) {
        // matrix_operations.cpp:797-799 (BatchedVector bvec(op.size(), op_ct); bvec.sum_elems_inplace(eval, gk)) and
        // the least-squares reductions (:919-928) through BatchedMatrix::sum_bvec_elems: every input ciphertext
        // as a batched vector of dimension <dim>; output 0 = bvec 0 summed out of place, then the matrix's bvecs
        const std::size_t dim = std::stoul(mode.substr(10));
        std::vector<BatchedVector> bvecs;
        for (auto &c : cts) bvecs.emplace_back(dim, c);
        keep.push_back(bvecs[0].sum_elems(eval, gk).get_bvec());
        BatchedMatrix m(BatchedMatrix::BatchingType::col, std::move(bvecs));
        BatchedMatrix s = m.sum_bvec_elems(eval, gk);
        for (const auto &b : s.get_bvecs()) keep.push_back(b.get_bvec());
    } else if (mode == "matrix_family") {
        // Matrix::left_matmul_with_transp, matmul_square, matmul_pow (he_linalg.cpp:241-349) on the first four
        // ciphertexts as a 2x2 column-major matrix, then matmul_pow(3), which needs operands of two levels
        // (A and A^2): SEAL throws there, and so must the drop-in (the last output is a marker)
        Matrix A(2, 2, std::vector<Ciphertext>(cts.begin(), cts.begin() + 4));
        for (const auto &m : {A.left_matmul_with_transp(eval, rk), A.matmul_square(eval, rk), A.matmul_pow(eval, rk, 2),
                              A.matmul_pow(eval, rk, 4)})
            for (const auto &c : m.get_elems()) keep.push_back(c);
        bool threw = false;
        try {
            (void)A.matmul_pow(eval, rk, 3);
        } catch (const std::invalid_argument &e) {
            threw = std::string(e.what()).find("mismatch") != std::string::npos;
        }
        keep.push_back(threw ? cts[0] : cts[1]);
    } else if (mode.rfind("math:", 0) == 0) {
        const std::size_t iter = std::stoul(mode.substr(5));
        hecdna::CKKSEncoder cencd(ctx);
        keep.push_back(he::math::signed_inv(cencd, eval, rk, cts[0], 1.0, iter));
        keep.push_back(he::math::inv_sqrt_twice(cencd, eval, rk, cts[0], 0.7, iter));
        keep.push_back(he::math::sqrt(ctx, cencd, eval, rk, cts[0], 1.0, iter));
        keep.push_back(he::math::abs(ctx, cencd, eval, rk, cts[1], 1.0, iter));
    } else if (mode == "util") {
        hecdna::CKKSEncoder cencd(ctx);
        Ciphertext d0 = cts[0];
        he::util::drop_chain_levels(ctx, cencd, eval, d0, 2);
        Ciphertext d1 = cts[1], d2 = cts[2];
        hecdna::Plaintext one_pt;
        he::util::reach_chain_level(ctx, cencd, eval, one_pt, std::vector<Ciphertext *>{&d1, &d2}, d0);
        for (const Ciphertext *c : {&d0, &d1, &d2})
            std::cout << "chain_index " << he::util::get_chain_index(ctx, *c) << " "
                      << he::util::get_chain_index(hecdna::EncryptionParameters(in.N, in.moduli), *c) << " "
                      << he::util::uint64_to_hex_string(c->parms_id()[0]) << "\n";
        keep.push_back(d0);
        keep.push_back(d1);
        keep.push_back(d2);
        // SEAL's chain walk (print_parameters, the chain loops of the examples): key level, then first .. last
        std::cout << "chain";
        for (auto cd = ctx.key_context_data(); cd; cd = cd->next_context_data()) std::cout << " " << cd->chain_index();
        std::cout << " first " << ctx.first_context_data()->chain_index() << " key_next "
                  << (ctx.key_context_data()->next_context_data() == ctx.first_context_data()) << "\n";
    } else if (mode == "least_squares") {
        // bench_he_least_squares_2d after encryption (matrix_operations.cpp:915-1003), x_ct = c0, y_ct = c1
        hecdna::CKKSEncoder cencd(ctx);
        const std::size_t n = 5;
        BatchedVector x_ctv(n, cts[0]);
        BatchedVector y_ctv(n, cts[1]);
        Ciphertext sum_x_ct = x_ctv.sum_elems(eval, gk).get_bvec();
        Ciphertext sum_y_ct = y_ctv.sum_elems(eval, gk).get_bvec();
        Ciphertext sum_xx_ct = x_ctv.square(eval, rk).sum_elems(eval, gk).get_bvec();
        Ciphertext sum_xy_ct = (eval % rk % x_ctv * y_ctv).sum_elems(eval, gk).get_bvec();
        hecdna::Plaintext n_pt;
        cencd.encode(n, sum_xx_ct.parms_id(), sum_xx_ct.scale(), n_pt);
        Ciphertext n_sum_xx_ct = eval % sum_xx_ct * n_pt;
        n_sum_xx_ct ^= eval;
        Ciphertext sum_x_sqr_ct;
        eval.square(sum_x_ct, sum_x_sqr_ct);
        sum_x_sqr_ct &= eval % rk;
        sum_x_sqr_ct ^= eval;
        hecdna::Plaintext one_pt;
        cencd.encode(1, sum_x_sqr_ct.parms_id(), sum_x_sqr_ct.scale(), one_pt);
        sum_x_sqr_ct *= eval % one_pt;
        sum_x_sqr_ct ^= eval;
        Ciphertext denom_ct = eval % n_sum_xx_ct - sum_x_sqr_ct;
        hecdna::Plaintext one_pt_;
        cencd.encode(std::vector<double>{1}, denom_ct.parms_id(), denom_ct.scale(), one_pt_);
        denom_ct *= eval % one_pt_;
        denom_ct ^= eval;
        Ciphertext denom_inv_ct = he::math::signed_inv(cencd, eval, rk, denom_ct, 0.05, 6);
        Ciphertext n_sum_xy_ct = eval % sum_xy_ct * n_pt;
        n_sum_xy_ct ^= eval;
        Ciphertext sum_x_sum_y_ct = eval % sum_x_ct * sum_y_ct;
        sum_x_sum_y_ct &= eval % rk;
        sum_x_sum_y_ct ^= eval;
        sum_x_sum_y_ct *= eval % one_pt;
        sum_x_sum_y_ct ^= eval;
        Ciphertext a_num_ct = eval % n_sum_xy_ct - sum_x_sum_y_ct;
        cencd.encode(1, sum_y_ct.parms_id(), sum_y_ct.scale(), one_pt);
        Ciphertext sum_y_sum_xx_ct = sum_y_ct;
        sum_y_sum_xx_ct *= eval % one_pt;
        sum_y_sum_xx_ct ^= eval;
        sum_y_sum_xx_ct *= eval % sum_xx_ct;
        sum_y_sum_xx_ct &= eval % rk;
        sum_y_sum_xx_ct ^= eval;
        Ciphertext sum_x_sum_xy_ct = sum_x_ct;
        sum_x_sum_xy_ct *= eval % one_pt;
        sum_x_sum_xy_ct ^= eval;
        sum_x_sum_xy_ct *= eval % sum_xy_ct;
        sum_x_sum_xy_ct &= eval % rk;
        sum_x_sum_xy_ct ^= eval;
        Ciphertext b_num_ct = eval % sum_y_sum_xx_ct - sum_x_sum_xy_ct;
        he::util::reach_chain_level(ctx, cencd, eval, one_pt, std::vector{&a_num_ct, &b_num_ct}, denom_inv_ct);
        Ciphertext a_ct = eval % a_num_ct * denom_inv_ct;
        a_ct &= eval % rk;
        a_ct ^= eval;
        Ciphertext b_ct = eval % b_num_ct * denom_inv_ct;
        b_ct &= eval % rk;
        b_ct ^= eval;
        for (Ciphertext *c : {&denom_ct, &denom_inv_ct, &a_num_ct, &b_num_ct, &a_ct, &b_ct}) keep.push_back(*c);
    } else if (mode == "matrix") {
        // Matrix::matmul on 2x2 element-wise ciphertext matrices (column-major elems)
        Matrix A(2, 2, std::vector<Ciphertext>(cts.begin(), cts.begin() + 4));
        Matrix B(2, 2, std::vector<Ciphertext>(cts.begin() + 4, cts.begin() + 8));
        Matrix C = A.matmul(eval, rk, B);
        for (const auto &c : C.get_elems()) keep.push_back(c);
    } else if (mode == "encode") {
        // matrix_operations.cpp:1079-1087: mat1[c][r] = 2 + dim c + r; each column replicated over the
        // slots as BatchedVector does; CKKSEncoder cencd(ctx); cencd.encode(mat1[i], scale, pt[i])
        const std::size_t dim = cts.size(), slots = ctx.slot_count();
        std::vector<std::vector<std::complex<double>>> mat1(dim, std::vector<std::complex<double>>(slots));
        int counter = 2;
        for (std::size_t c = 0; c < dim; ++c) {
            for (std::size_t r = 0; r < slots; ++r) mat1[c][r] = std::complex<double>(counter + r % dim, 0);
            counter += (int)dim;
        }
        hecdna::CKKSEncoder cencd(ctx);
        std::vector<hecdna::Plaintext> pts(dim);
        for (std::size_t i = 0; i + 1 < dim; ++i) cencd.encode(mat1[i], std::pow(2.0, 40), pts[i]);
        std::vector<double> lastcol(slots);  // the last column through the batched real-valued form
        for (std::size_t r = 0; r < slots; ++r) lastcol[r] = mat1[dim - 1][r].real();
        std::vector<hecdna::Plaintext> last;
        cencd.encode_batch({lastcol}, std::pow(2.0, 40), last);
        pts[dim - 1] = last[0];
        std::ofstream f(argv[3], std::ios::binary);
        const std::uint64_t n = dim;
        f.write(reinterpret_cast<const char *>(&n), 8);
        for (const auto &p : pts) {
            const std::uint64_t s = 1, l = p.level();
            const double sc = p.scale();
            const auto d = p.download();
            f.write(reinterpret_cast<const char *>(&s), 8);
            f.write(reinterpret_cast<const char *>(&l), 8);
            f.write(reinterpret_cast<const char *>(&sc), 8);
            f.write(reinterpret_cast<const char *>(d.data()), d.size() * 8);
        }
        std::cout << "he_demo encode: wrote " << dim << " plaintexts\n";
        return 0;
    } else {
        std::cout << "No such demo for " << mode << ".\n";
        return 1;
    }
    for (auto &c : keep) outs.push_back(&c);
    write_output(argv[3], outs);
    std::cout << "he_demo " << mode << ": wrote " << outs.size() << " ciphertexts\n";
    return 0;
}
