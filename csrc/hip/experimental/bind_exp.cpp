// pybind11 module `_onihip_exp`: E-step variants measured NOT faster than the shipped kernels, kept
// buildable for their oracle tests and benchmarks but outside `_onihip` (ml_ops never loads them).
//
//   gs_xsplit -- one document over the CUs of one XCD (profiles/r5_xcd_split.md: 1.52 ms for the
//                headline day's longest document vs 1.48-1.49 ms on one workgroup)
#include <pybind11/pybind11.h>

#include "common.h"
#include "kernels.h"

namespace py = pybind11;
using u = uintptr_t;

template <typename T>
static T* P(u x) {
  return reinterpret_cast<T*>(x);
}
static hipStream_t S(u x) { return reinterpret_cast<hipStream_t>(x); }

PYBIND11_MODULE(_onihip_exp, m) {
  m.doc() = "oni_ml_amd experimental gfx950 E-step kernels (not used by ml_ops)";
  m.def("gs_xsplit_rows", [](int KS) { return oni::gs_xsplit_rows(KS); });
  m.def("gs_xsplit", [](u doc_ptr, u word_idx, u counts, u beta, int K, int KS, int gs_updates, u params, u gamma,
                        u cphi, u lik, u alpha_ss, u iters, u seg_doc, u seg_index, u seg_count, u seg_base,
                        u doc_slot, int n_blocks, int n_rows, u xchg, u counter, int n_docs, u error, int proto,
                        u placed, u stream, u dbg) {
    oni::GSArgs a{P<const int>(doc_ptr), P<const int>(word_idx), P<const float>(counts), nullptr,
                  n_blocks,              P<const double>(beta),  K,                      gs_updates,
                  P<const double>(params), P<double>(gamma),     P<double>(cphi),        P<double>(lik),
                  P<double>(alpha_ss),   P<int>(iters),         P<long long>(dbg)};
    oni::XSplitArgs s{P<const int>(seg_doc), P<const int>(seg_index), P<const int>(seg_count),
                      P<const int>(seg_base), P<const int>(doc_slot), n_blocks, n_rows,
                      P<unsigned>(xchg), P<int>(counter), n_docs, P<int>(error), proto, P<int>(placed)};
    oni::launch_gs_xsplit(a, s, KS, S(stream));
  });
}
