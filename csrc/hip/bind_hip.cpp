// pybind11 module `_onihip`: thin launch bindings for the gfx950 kernels.
//
// Arguments are raw device addresses (torch tensor .data_ptr()) and the HIP
// stream handle of the caller (torch.cuda.current_stream().cuda_stream), so
// launches join torch's stream order and can be captured into hipGraphs.
// Shape/dtype/contiguity validation happens in oni_ml_amd/ops/hip.py before
// any launch.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <tuple>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace py = pybind11;
using u = uintptr_t;

template <typename T>
static T* P(u x) {
  return reinterpret_cast<T*>(x);
}
static hipStream_t S(u x) { return reinterpret_cast<hipStream_t>(x); }

PYBIND11_MODULE(_onihip, m) {
  m.doc() = "oni_ml_amd CDNA4 (gfx950) HIP kernels";

  m.def("compiled_ks", []() {
    std::vector<int> v;
#define ONI_KS(X) v.push_back(X);
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    return v;
  });

  m.def("device_name", []() {
    hipDeviceProp_t p;
    int dev = 0;
    ONI_HIP_CHECK(hipGetDevice(&dev));
    ONI_HIP_CHECK(hipGetDeviceProperties(&p, dev));
    return std::string(p.gcnArchName);
  });

  m.def("suff_fused_blocks", [](int h, int m_, int l) { return oni::suff_fused_blocks(h, m_, l); });
  m.def("rows_accumulate", [](u rows, u ptr, u src, u own, u recv, u out, int n_rows, int width, u stream) {
    oni::launch_rows_accumulate(P<const int>(rows), P<const int>(ptr), P<const int>(src), P<const double>(own),
                                P<const double>(recv), P<double>(out), n_rows, width, S(stream));
  });
  m.def("log_beta_t", [](u cw, int V, int K, int ld, u ct, double floor_v, u out, u stream) {
    oni::launch_log_beta_t(P<const double>(cw), V, K, ld, P<const double>(ct), floor_v, P<double>(out), S(stream));
  });
  m.def("colsum_partials", [](u part, int nb, int cols, u out, u gate, u stream) {
    oni::launch_colsum_partials(P<const double>(part), nb, cols, P<double>(out), P<const double>(gate), S(stream));
  });
  m.def("em_control", [](u scalars, u params, u ctl, u hist, int hist_slots, u stream) {
    oni::launch_em_control(P<const double>(scalars), P<double>(params), P<double>(ctl), P<double>(hist), hist_slots,
                           S(stream));
  });
  m.def("param_count", []() { return oni::kParamCount; });
  m.def("hist_cols", []() { return oni::kHistCols; });

  m.def("alpha_newton", [](u scalars, double num_docs, int K, bool estimate, u params, u alpha_out, u stream) {
    oni::launch_alpha_newton(P<const double>(scalars), num_docs, K, estimate, P<double>(params), P<double>(alpha_out),
                             S(stream));
  });


  // ---------------------------------------------- fp64 block Gauss-Seidel ---
  m.def("gs_umax", [](int KS) { return KS > 0 ? oni::gs_umax(KS) : oni::kGsUMax; }, py::arg("KS") = 0);
  m.def("gs_tiny_max", [](int KS) { return oni::gs_tiny_max(KS); });
  m.def("gs_estep", [](u doc_ptr, u word_idx, u counts, u order, int n_items, u beta, int K, int KS, int gs_updates,
                       u params, u gamma, u cphi, u lik, u alpha_ss, u iters, int variant, u stream, u dbg,
                       u stage, u stage_off) {
    oni::GSArgs a{P<const int>(doc_ptr), P<const int>(word_idx), P<const float>(counts), P<const int>(order),
                  n_items,               P<const double>(beta),  K,                      gs_updates,
                  P<const double>(params), P<double>(gamma),     P<double>(cphi),        P<double>(lik),
                  P<double>(alpha_ss),   P<int>(iters),         P<long long>(dbg),      P<const double>(stage),
                  P<const long long>(stage_off)};
    oni::launch_gs_estep(a, variant, KS, S(stream));
  });
  m.def("gs_stage", [](u beta, u word_idx, u tile_ent, u tile_cnt, int n_tiles, u stage, int KS, u gate, u stream) {
    oni::launch_gs_stage(P<const double>(beta), P<const int>(word_idx), P<const int>(tile_ent),
                         P<const int>(tile_cnt), n_tiles, P<double>(stage), KS, P<const double>(gate), S(stream));
  });
  m.def("init_random_ss", [](u cw, int V, int K, int KS, unsigned long long seed, u stream) {
    oni::launch_init_random_ss(P<double>(cw), V, K, KS, seed, S(stream));
  });
  m.def("gs_split_capacity", [](int KS) { return oni::gs_split_capacity(KS); });
  m.def("gs_split_umax", [](int KS) { return oni::gs_split_umax(KS); });
  m.def("gs_split_lds_umax", [](int KS) { return oni::gs_split_lds_umax(KS); });
  m.def("gs_split", [](u doc_ptr, u word_idx, u counts, u beta, int K, int KS, int gs_updates, u params, u gamma,
                       u cphi, u lik, u alpha_ss, u iters, u seg_doc, u seg_index, u seg_count, u seg_base,
                       u doc_slot, int n_blocks, u xchg, u counter, int n_docs, u error, u stream, u dbg, u tab,
                       int tab_rows, u csum, int csum_stride) {
    oni::GSArgs a{P<const int>(doc_ptr), P<const int>(word_idx), P<const float>(counts), nullptr,
                  n_blocks,              P<const double>(beta),  K,                      gs_updates,
                  P<const double>(params), P<double>(gamma),     P<double>(cphi),        P<double>(lik),
                  P<double>(alpha_ss),   P<int>(iters),         P<long long>(dbg)};
    oni::SplitArgs s{P<const int>(seg_doc), P<const int>(seg_index), P<const int>(seg_count),
                     P<const int>(seg_base), P<const int>(doc_slot), n_blocks, tab_rows,
                     P<unsigned long long>(xchg), P<int>(counter), n_docs, P<int>(error), P<double>(tab),
                     P<const double>(csum), csum_stride};
    oni::launch_gs_split(a, s, KS, S(stream));
  });
  m.def("gs_suff64", [](u word_ptr, u csc_ent, u order, int n_heavy, int n_medium, int n_light, u cphi, u cw, u part,
                        u lik, u ass, int lo, int hi, int KS, u gate, u stream, u cw_base) {
    oni::launch_gs_suff64(P<const int>(word_ptr), P<const int>(csc_ent), P<const int>(order), n_heavy, n_medium,
                          n_light, P<const double>(cphi), P<double>(cw), P<double>(part), P<const double>(lik),
                          P<const double>(ass), lo, hi, KS, P<const double>(gate), S(stream),
                          P<const double>(cw_base));
  });
  m.def("gs_mstep_control", [](u cw, u class_total, u beta, int V, int K, int KS, u scalars, u params, u ctl,
                               u hist, int hist_slots, u done_count, u stream, u rows, int n_rows, int newton,
                               int estimate, double num_docs, u alpha_out, u st_word_idx,
                               std::vector<std::tuple<u, u, u, int>> st_sets) {
    oni::EMControlArgs c{P<const double>(scalars), P<double>(params), P<double>(ctl), P<double>(hist), hist_slots,
                         P<int>(done_count)};
    const oni::NewtonArgs nw{newton, estimate, num_docs, P<double>(alpha_out)};
    if (newton && !alpha_out) throw std::runtime_error("gs_mstep_control: alpha_out required with newton");
    oni::StageFuseArgs sf;
    if (st_sets.size() > 2) throw std::runtime_error("gs_mstep_control: at most 2 staged sets");
    sf.word_idx = P<const int>(st_word_idx);
    for (const auto& [ent, cnt, out, n] : st_sets) {
      sf.tile_ent[sf.n_sets] = P<const int>(ent);
      sf.tile_cnt[sf.n_sets] = P<const int>(cnt);
      sf.out[sf.n_sets] = P<double>(out);
      sf.n_tiles[sf.n_sets] = n;
      ++sf.n_sets;
    }
    oni::launch_gs_mstep_control(P<const double>(cw), P<const double>(class_total), P<double>(beta), V, K, KS,
                                 P<const int>(rows), n_rows, c, nw, S(stream), sf);
  }, py::arg("cw"), py::arg("class_total"), py::arg("beta"), py::arg("V"), py::arg("K"), py::arg("KS"),
     py::arg("scalars"), py::arg("params"), py::arg("ctl"), py::arg("hist"), py::arg("hist_slots"),
     py::arg("done_count"), py::arg("stream"), py::arg("rows"), py::arg("n_rows"), py::arg("newton"),
     py::arg("estimate"), py::arg("num_docs"), py::arg("alpha_out"), py::arg("st_word_idx") = 0,
     py::arg("st_sets") = std::vector<std::tuple<u, u, u, int>>());
  m.def("gs_mstep", [](u cw, u class_total, u beta, int V, int K, int KS, u gate, u stream) {
    oni::launch_gs_mstep(P<const double>(cw), P<const double>(class_total), P<double>(beta), V, K, KS,
                         P<const double>(gate), S(stream));
  });

  m.def("score_events", [](u theta, u phi, int K, double dflt, u doc_a, u word_a, u doc_b, u word_b,
                           int64_t n, double tol, u score_a, u score_b, u key, u flag, u stream) {
    oni::ScoreArgs a{P<const double>(theta), P<const double>(phi), K, dflt,
                     P<const int>(doc_a),    P<const int>(word_a), P<const int>(doc_b),
                     P<const int>(word_b),   n,                    tol,
                     P<double>(score_a),     P<double>(score_b),   P<double>(key),
                     P<uint8_t>(flag)};
    oni::launch_score_events(a, S(stream));
  });

  m.def("flow_words", [](u hour, u minute, u second, u port_a, u port_b, u ipkt, u ibyt, u time_cuts,
                         int n_time, u ibyt_cuts, int n_ibyt, u ipkt_cuts, int n_ipkt, int64_t n, u time_out,
                         u time_bin, u ibyt_bin, u ipkt_bin, u word_port, u p_case, u src_prefix,
                         u dst_prefix, u stream) {
    oni::FlowWordArgs a{};
    a.hour = P<const double>(hour);
    a.minute = P<const double>(minute);
    a.second = P<const double>(second);
    a.port_a = P<const double>(port_a);
    a.port_b = P<const double>(port_b);
    a.ipkt = P<const double>(ipkt);
    a.ibyt = P<const double>(ibyt);
    a.time_cuts = P<const double>(time_cuts);
    a.ibyt_cuts = P<const double>(ibyt_cuts);
    a.ipkt_cuts = P<const double>(ipkt_cuts);
    a.n_time_cuts = n_time;
    a.n_ibyt_cuts = n_ibyt;
    a.n_ipkt_cuts = n_ipkt;
    a.n = n;
    a.time_out = P<double>(time_out);
    a.time_bin = P<int8_t>(time_bin);
    a.ibyt_bin = P<int8_t>(ibyt_bin);
    a.ipkt_bin = P<int8_t>(ipkt_bin);
    a.word_port = P<double>(word_port);
    a.p_case = P<int8_t>(p_case);
    a.src_prefix = P<int8_t>(src_prefix);
    a.dst_prefix = P<int8_t>(dst_prefix);
    oni::launch_flow_words(a, S(stream));
  });

  m.def("bin_columns", [](std::vector<u> values, std::vector<u> cuts, std::vector<int> ncuts, int64_t n,
                          u bins, u stream) {
    if (values.size() != cuts.size() || values.size() != ncuts.size())
      throw std::runtime_error("bin_columns: column lists differ in length");
    std::vector<const double*> v, c;
    for (auto x : values) v.push_back(P<const double>(x));
    for (auto x : cuts) c.push_back(P<const double>(x));
    oni::launch_bin_columns(v.data(), c.data(), ncuts.data(), (int)values.size(), n, P<int8_t>(bins),
                            S(stream));
  });
}
