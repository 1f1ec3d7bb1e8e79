// Host symbolic analysis for the supernodal multifrontal factorization.
//
// Reference counterparts (evanwporter/SparseCholesky):
//   etree            include/chol.hpp:377-410
//   post_order/tdfs  include/chol.hpp:445-499
//   col_count        include/chol.hpp:506-622
//   ereach           include/chol.hpp:680-739
//   schol            include/chol.hpp:873-946
//   compute_levels / compute_supernodes / atree   src/chol.cpp:7-136
//
// The numeric plan works in etree postorder ("internal" numbering) so that
// every supernode is a contiguous range of columns.  A postorder is a
// topological order of the etree, so the factor of P A P^T is P L P^T with
// the same values; export maps back to the natural numbering.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/sparsecholesky.h"

namespace sc {

using i32 = int32_t;
using i64 = int64_t;

// ---- reference-API helpers (natural numbering) ----
void etree(i64 n, const i64* Ap, const i32* Ai, i32* parent);
void post_order(i64 n, const i32* parent, i32* post);
void col_count(i64 n, const i64* Ap, const i32* Ai, const i32* parent, const i32* post,
               i64* colcount);
i64 ereach(i64 n, const i64* Ap, const i32* Ai, const double* Ax, i64 k, const i32* parent,
           i32* s, i32* w, double* x, std::vector<i32>& path);
i64 compute_levels(i64 n, const i32* parent, i32* level_of);
i64 etree_depth(i64 n, const i32* parent);

// Front size classes
enum FrontClass : int32_t { FRONT_SMALL = 0, FRONT_LARGE = 1 };

constexpr int kAsmRows = 256;  // row tile of the large-front assembly (kernels.hpp ASM_ROWS)
constexpr int kAsmCols = 16;   // column block of the large-front assembly (kernels.hpp ASM_COLS)

struct Symbolic {
    sc_options opt {};
    i64 n = 0;
    i64 nnzA_in = 0;   // entries in the input arrays (incl. ignored lower ones)
    i64 nnzA_used = 0; // upper entries actually used
    std::vector<i64> Ap;  // copy of input pattern (natural)
    std::vector<i32> Ai;

    // natural-order symbolic (reference semantics)
    std::vector<i32> perm;      // fill-reducing ordering, new -> old (empty: the given order)
    std::vector<i32> parent;    // etree
    std::vector<i32> post;      // internal -> natural
    std::vector<i32> ipost;     // natural -> internal
    std::vector<i64> colcount;  // natural numbering
    i64 nnzL = 0;
    double flops = 0.0;
    i64 depth = 0;

    // supernodes, internal numbering
    i64 n_fundamental = 0;
    i32 ns = 0;
    std::vector<i32> sn_start;   // ns+1
    std::vector<i32> sn_of;      // internal column -> supernode
    std::vector<i32> sn_m;       // front rows
    std::vector<i64> rows_ptr;   // ns+1
    std::vector<i32> rows;       // internal row indices, ascending; first w are the pivots
    std::vector<i32> sn_parent;
    std::vector<i32> child_ptr;  // ns+1
    std::vector<i32> child_list;
    std::vector<i64> rel_ptr;    // ns+1, CB row -> position in parent front
    std::vector<i32> relind;
    // per child: bounds of its CB rows by blocks of the parent front, compact over the
    // blocks it touches (symbolic.cpp bounds(), kernels.hip bnd_at): the assembly's
    // kAsmRows-row tiles (rel_bnd), kAsmCols-column blocks (col_bnd), and the 64-row
    // blocks of the parent's contribution block (tile_bnd, the CB SYRK's extend-add gather)
    std::vector<i64> rb_ptr;     // ns+1
    std::vector<i32> rel_bnd;
    std::vector<i64> cbk_ptr;    // ns+1
    std::vector<i32> col_bnd;
    std::vector<i64> tb_ptr;     // ns+1
    std::vector<i32> tile_bnd;
    std::vector<i64> panel_off;  // ns+1 (doubles), L panel m x w, ld = m
    std::vector<i64> cb_off;     // ns+1 (doubles), CB mb x mb, ld = mb
    std::vector<i64> a_ptr;      // n+1: A entries grouped by internal column (lower part)
    std::vector<i32> a_pos;      // row position of the entry inside its column's front
    std::vector<i64> a_src;      // index of the entry in the input arrays
    std::vector<i32> level;      // assembly-tree height: leaves 0
    i32 nlevels = 0;
    std::vector<i32> fclass;     // FrontClass per supernode

    // statistics
    sc_symbolic_stats stats {};

    i32 w(i32 s) const { return sn_start[s + 1] - sn_start[s]; }
    i32 m(i32 s) const { return sn_m[s]; }
    i32 mb(i32 s) const { return sn_m[s] - w(s); }
};

// Build the symbolic analysis.  Returns SC_OK or an sc_status error; on error
// `err` holds a message.
i64 analyze(i64 n, const i64* Ap, const i32* Ai, const sc_options& opt, Symbolic& S,
            std::string& err);

// Fill-reducing ordering (ordering.cpp): nested dissection by level structures,
// perm[new] = old; and B = P A P^T as upper CSC with src[q] = A-index of entry q.
i64 nd_order(i64 n, const i64* Ap, const i32* Ai, i32* perm);
// Approximate minimum degree ordering (ordering.cpp), perm[new] = old.
i64 amd_order(i64 n, const i64* Ap, const i32* Ai, i32* perm);
void permute_upper(i64 n, const i64* Ap, const i32* Ai, const i32* perm, std::vector<i64>& Bp,
                   std::vector<i32>& Bi, std::vector<i64>& src);

// Reference-layout pattern of L (schol().p()/i()), natural numbering.
void pattern_L(const Symbolic& S, i64* Lp, i32* Li);

// Export: supernodal panels (host copy of the gathered panels; supernode s at
// panels + poff[s], m x w, ld = m) -> reference CSC.
void export_L(const Symbolic& S, const double* panels, const i64* poff, i64* Lp, i32* Li, double* Lx);

}  // namespace sc
