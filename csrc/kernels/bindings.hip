// pybind11 launch bindings of the gfx950 kernels (_hipk). Arguments arrive as a dict of
// device pointers (torch data_ptr()) and sizes; igaming_platform_amd/ops/kernels.py builds
// the dicts and validates every shape/dtype/device before calling in.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>
#include <string>
#include <vector>

#include "launch.h"
#include "update.h"
#include "oplist.h"

namespace py = pybind11;
using namespace igp;

namespace {

template <class T>
T ptr(const py::dict& d, const char* k) {
  if (!d.contains(k)) return nullptr;
  py::object o = d[k];
  if (o.is_none()) return nullptr;
  return reinterpret_cast<T>(o.cast<uintptr_t>());
}

int32_t geti(const py::dict& d, const char* k, int32_t def = 0) {
  if (!d.contains(k)) return def;
  return d[k].cast<int32_t>();
}

hipStream_t stream_of(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

EnsembleArgs ensemble_args(const py::dict& d) {
  EnsembleArgs a{};
  a.hdr = ptr<const BatchHdr*>(d, "hdr");
  a.cfg = ptr<const ScoreCfg*>(d, "cfg");
  a.feat = ptr<const FeatRec*>(d, "feat");
  a.X = ptr<const float*>(d, "X");
  a.x_stride = geti(d, "x_stride");
  a.ml = ptr<const float*>(d, "ml");
  a.out = ptr<ResultRec*>(d, "out");
  a.host_out = ptr<ResultRec*>(d, "host_out");
  a.metrics = ptr<unsigned long long*>(d, "metrics");
  a.n_rows = geti(d, "n_rows");
  a.route = ptr<const int32_t*>(d, "route");
  a.route_c = geti(d, "route_c");
  a.route_stride = geti(d, "route_stride");
  if (a.route && (!a.host_out || a.route_c < 1 || a.route_stride < a.route_c * (int)sizeof(ResultRec)))
    throw std::runtime_error("ensemble: routed host rows need host_out, route_c and route_stride");
  return a;
}

UpdateArgs update_args(const py::dict& d) {
  UpdateArgs a{};
  a.cfg = ptr<const ScoreCfg*>(d, "cfg");
  a.hdr = ptr<const BatchHdr*>(d, "hdr");
  a.n = geti(d, "n");
  a.n_max = geti(d, "n_max");
  a.req = ptr<const ReqRec*>(d, "req");
  a.ring_ts = ptr<uint32_t*>(d, "ring_ts");
  a.ring_amt = ptr<int64_t*>(d, "ring_amt");
  a.hll = ptr<uint8_t*>(d, "hll");
  a.rt = ptr<AcctRT*>(d, "rt");
  a.ev = ptr<uint16_t*>(d, "ev");
  a.ring_size = geti(d, "ring_size");
  a.ev_ring = geti(d, "ev_ring");
  a.ev_dim = geti(d, "ev_dim");
  a.dbuf = ptr<int32_t*>(d, "dbuf");
  a.dcap = geti(d, "dcap");
  a.dmax = geti(d, "dmax");
  a.region = geti(d, "region", DEDUP_STANDALONE);
  a.src = ptr<const char*>(d, "src");
  a.hll_lc = ptr<const int32_t*>(d, "hll_lc");
  if (!a.hll_lc) throw std::runtime_error("update args: hll_lc table required (cached HLL estimates)");
  a.xrecv = ptr<const ReqRec*>(d, "xrecv");
  a.route = ptr<int32_t*>(d, "route");
  a.xhdr = ptr<const int4*>(d, "xhdr");
  a.xn = geti(d, "xn");
  a.xc = geti(d, "xc");
  a.xpstride = geti(d, "xpstride");
  if (a.xrecv && (a.src || !a.route || !a.xhdr || a.xn < 1 || a.xn > 64 || a.xc < 1 || a.xpstride < a.xc + 1 ||
                  a.xn * a.xc > a.n_max || a.region >= 0 || !a.hdr))
    throw std::runtime_error("update args: rows-region source (xrecv, route, xhdr, 1 <= xn <= 64, xc, stride)");
  if (a.src && (a.region >= 0 || !a.hdr)) throw std::runtime_error("update args: slab source needs the scorer ring");
  if (!a.dbuf || !a.cfg || !a.req || !a.rt) throw std::runtime_error("update args: missing pointers");
  if (a.n_max > a.dmax || a.dcap < 2 * a.dmax) throw std::runtime_error("update args: dedup scratch too small");
  if (a.ev && a.ev_dim != 16) throw std::runtime_error("update args: event dim must be 16");
  if (a.region < 0 && !a.hdr) throw std::runtime_error("update args: ring region needs hdr");
  if (a.region > DEDUP_STANDALONE) throw std::runtime_error("update args: bad dedup region");
  return a;
}

void check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// launch now on stream s, or (record mode, oplist.h) append the launch to the list being built
template <class F>
void launch_or_record(F f, uintptr_t s, const char* what) {
  if (OpList* r = recording()) {
    r->ops.emplace_back(std::move(f));
    return;
  }
  f(stream_of(s));
  check(what);
}

}  // namespace

namespace igp {
OpList*& recording() {
  thread_local OpList* cur = nullptr;
  return cur;
}
StopEvent& stop_event() {
  thread_local StopEvent se;
  return se;
}
}  // namespace igp

namespace igp {
void register_driver(py::module_& m);
void register_model_driver(py::module_& m);
void register_exchange(py::module_& m);
void register_watch(py::module_& m);
}

PYBIND11_MODULE(_hipk, m) {
  m.doc() = "igaming_platform_amd gfx950 HIP kernels";
  m.attr("ARCH") = "gfx950";
  m.attr("SIZEOF_SCORECFG") = (int)sizeof(ScoreCfg);
  m.attr("SIZEOF_FEATREC") = (int)sizeof(FeatRec);
  m.attr("SIZEOF_ACCTRT") = (int)sizeof(AcctRT);
  m.attr("SIZEOF_ACCTBATCH") = (int)sizeof(AcctBatch);
  m.attr("SIZEOF_REQREC") = (int)sizeof(ReqRec);
  m.attr("DEDUP_LIST") = DEDUP_LIST;
  m.attr("DEDUP_REGIONS") = DEDUP_RING + 1;
  m.def("dedup_region_size", [](int cap, int n_max) { return (int64_t)dedup_region_size(cap, n_max); });
  igp::register_driver(m);
  igp::register_model_driver(m);
  igp::register_exchange(m);
  igp::register_watch(m);

  m.def("feature_assemble", [](py::dict d, uintptr_t s) {
    AssembleArgs a{};
    a.hdr = ptr<const BatchHdr*>(d, "hdr");
    a.cfg = ptr<const ScoreCfg*>(d, "cfg");
    a.req = ptr<const ReqRec*>(d, "req");
    a.ring_ts = ptr<const uint32_t*>(d, "ring_ts");
    a.ring_amt = ptr<const int64_t*>(d, "ring_amt");
    a.hll = ptr<const uint8_t*>(d, "hll");
    a.rt = ptr<const AcctRT*>(d, "rt");
    a.batch = ptr<const AcctBatch*>(d, "batch");
    a.ext = ptr<const float*>(d, "ext");
    a.bl_keys = ptr<const uint64_t*>(d, "bl_keys");
    a.bl_exp = ptr<const uint32_t*>(d, "bl_exp");
    a.ip_keys = ptr<const uint64_t*>(d, "ip_keys");
    a.ip_flags = ptr<const uint32_t*>(d, "ip_flags");
    a.hll_lc = ptr<const int32_t*>(d, "hll_lc");
    if (!a.hll_lc) throw std::runtime_error("feature_assemble: hll_lc table required");
    a.X = ptr<float*>(d, "X");
    a.feat = ptr<FeatRec*>(d, "feat");
    a.fenc = ptr<uint8_t*>(d, "fenc");
    a.fenc_route = ptr<const int32_t*>(d, "fenc_route");
    a.fenc_c = geti(d, "fenc_c");
    a.fenc_stride = geti(d, "fenc_stride");
    if (a.fenc_route && (!a.fenc || a.fenc_c < 1 || a.fenc_stride < a.fenc_c * (int)sizeof(FeatRec)))
      throw std::runtime_error("feature_assemble: routed images need fenc, fenc_c and fenc_stride");
    a.dbuf = ptr<int32_t*>(d, "dbuf");
    a.dcap = geti(d, "dcap");
    a.dmax = geti(d, "dmax");
    a.x_stride = geti(d, "x_stride");
    a.ring_size = geti(d, "ring_size");
    a.n_rows = geti(d, "n_rows");
    if (a.dbuf) {
      if (!d.contains("upd")) throw std::runtime_error("feature_assemble: score-then-update needs upd args");
      a.upd = update_args(d["upd"].cast<py::dict>());
      if (a.upd.region >= 0 || a.upd.dbuf != a.dbuf) throw std::runtime_error("feature_assemble: upd region");
    }
    a.trace = ptr<int64_t*>(d, "trace");
    launch_or_record([a](hipStream_t st) { launch_feature_assemble(a, st); }, s, "feature_assemble");
  });

  // record mode (oplist.h): launches between record_begin() and record_end() are stored, not run
  py::class_<OpList, std::shared_ptr<OpList>>(m, "OpList")
      .def_property_readonly("size", [](const OpList& o) { return o.ops.size(); })
      .def("run", [](const OpList& o, uintptr_t s) {  // issue the recorded launches on stream s
        py::gil_scoped_release nogil;
        o.run(stream_of(s));
        check("OpList.run");
      });
  m.def("record_begin", []() {
    if (recording()) throw std::runtime_error("record_begin: already recording on this thread");
    recording() = new OpList();
  });
  m.def("record_end", []() {
    OpList* r = recording();
    if (!r) throw std::runtime_error("record_end: not recording");
    recording() = nullptr;
    return std::shared_ptr<OpList>(r);
  });
  // stream-ordered copy between pinned host and device memory (recordable)
  m.def("memcpy_async", [](uintptr_t dst, uintptr_t src, size_t n, uintptr_t s) {
    if (!dst || !src) throw std::runtime_error("memcpy_async: null pointer");
    launch_or_record([dst, src, n](hipStream_t st) {
      const hipError_t e = hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n,
                                          hipMemcpyDefault, st);
      if (e != hipSuccess) throw std::runtime_error(std::string("memcpy_async: ") + hipGetErrorString(e));
      stop_event().bound = false;  // a copy after the stage's last kernel: the driver records the event
    }, s, "memcpy_async");
  });

  // a stream whose kernels run only on the CUs set in `mask` (32 CUs per word): lets the
  // scorer keep its state and model streams on disjoint CUs (tools: IGP_CU_SPLIT)
  m.def("cu_stream", [](std::vector<uint32_t> mask) {
    hipStream_t st = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data());
    if (e != hipSuccess) throw std::runtime_error(std::string("hipExtStreamCreateWithCUMask: ") + hipGetErrorString(e));
    return reinterpret_cast<uintptr_t>(st);
  });

  m.def("cu_stream_destroy", [](uintptr_t st) {
    const hipError_t e = hipStreamDestroy(reinterpret_cast<hipStream_t>(st));
    if (e != hipSuccess) throw std::runtime_error(std::string("hipStreamDestroy: ") + hipGetErrorString(e));
  });

  m.def("feature_update", [](py::dict d, uintptr_t s) {
    UpdateArgs a = update_args(d);
    const int mode = geti(d, "segments_only") ? 1 : geti(d, "insert_only") ? 2 : 0;
    launch_or_record([a, mode](hipStream_t st) {
      if (mode == 1) launch_update_segments(a, st);
      else if (mode == 2) launch_dedup_insert(a, st);
      else launch_feature_update(a, st);
    }, s, "feature_update");
  });

  auto tree_args = [](const py::dict& d) {
    TreeArgs a{};
    a.hdr = ptr<const BatchHdr*>(d, "hdr");
    a.X = ptr<const float*>(d, "X");
    a.nodes = ptr<const float2*>(d, "nodes");
    a.leaves = ptr<const float*>(d, "leaves");
    a.base = ptr<const float*>(d, "base");
    a.out = ptr<float*>(d, "out");
    a.x_stride = geti(d, "x_stride");
    a.n_rows = geti(d, "n_rows");
    a.n_trees = geti(d, "n_trees");
    a.depth = geti(d, "depth");
    a.k = geti(d, "k");
    a.n_out = geti(d, "n_out");
    a.post = geti(d, "post");
    a.average = geti(d, "average");
    a.binary_class = geti(d, "binary_class", -1);
    a.all_positive = geti(d, "all_positive", 1);
    a.no_finish = geti(d, "no_finish", 0);
    a.all_leq = geti(d, "all_leq", 0);
    a.trace = ptr<int64_t*>(d, "trace");
    return a;
  };

  m.def("tree_ensemble", [tree_args](py::dict d, uintptr_t s) {
    TreeArgs a = tree_args(d);
    const int groups = geti(d, "groups", 1);
    float* partial = ptr<float*>(d, "partial");
    if (d.contains("ens") && !d["ens"].is_none()) {
      // K5 fused into the finish kernel: only a grouped launch has one
      if (groups <= 1 || !partial || a.no_finish) throw std::runtime_error("tree_ensemble: ensemble fusion needs a grouped launch");
      a.fuse_ens = 1;
      a.ens = ensemble_args(d["ens"].cast<py::dict>());
      if (!a.ens.hdr || !a.ens.cfg || !a.ens.feat || !a.ens.out || a.ens.ml != a.out)
        throw std::runtime_error("tree_ensemble: ensemble args (ml must be the tree output)");
    }
    launch_or_record([a, groups, partial](hipStream_t st) { launch_tree_ensemble_grouped(a, groups, partial, st); },
                     s, "tree_ensemble");
  });

  m.def("tree_sparse", [](py::dict d, uintptr_t s) {
    TreeSparseArgs a{};
    a.X = ptr<const float*>(d, "X");
    a.nodes = ptr<const int32_t*>(d, "nodes");
    a.roots = ptr<const int32_t*>(d, "roots");
    a.leaf_w = ptr<const float*>(d, "leaf_w");
    a.leaf_has = ptr<const uint8_t*>(d, "leaf_has");
    a.base = ptr<const float*>(d, "base");
    a.out = ptr<float*>(d, "out");
    a.x_stride = geti(d, "x_stride");
    a.n_rows = geti(d, "n_rows");
    a.n_trees = geti(d, "n_trees");
    a.depth = geti(d, "depth");
    a.k = geti(d, "k");
    a.n_out = geti(d, "n_out");
    a.post = geti(d, "post");
    a.aggregate = geti(d, "aggregate");
    a.binary_class = geti(d, "binary_class", -1);
    a.all_positive = geti(d, "all_positive", 1);
    a.feat_w = geti(d, "feat_w");
    const int groups = geti(d, "groups", 1);
    float* partial = ptr<float*>(d, "partial");
    if (!a.X || !a.nodes || !a.roots || !a.leaf_w || !a.leaf_has || !a.out) throw std::runtime_error("tree_sparse: args");
    if (a.k < 1 || a.k > 64) throw std::runtime_error("tree_sparse: 1..64 targets");
    if (a.post < 0 || a.post > 4 || a.aggregate < 0 || a.aggregate > 3) throw std::runtime_error("tree_sparse: post/aggregate");
    if (a.feat_w < 1 || a.feat_w > a.x_stride) throw std::runtime_error("tree_sparse: feature width");
    if (a.depth < 0 || a.depth > 4096) throw std::runtime_error("tree_sparse: depth");
    if (groups < 1 || (groups > 1 && !partial)) throw std::runtime_error("tree_sparse: grouped launch needs partial");
    if (a.binary_class >= 0 ? a.n_out != 2 : a.n_out != a.k) throw std::runtime_error("tree_sparse: n_out");
    launch_or_record([a, groups, partial](hipStream_t st) { launch_tree_sparse(a, groups, partial, st); }, s,
                     "tree_sparse");
  });

  auto gemm_args = [](const py::dict& d) {
    GemmArgs a{};
    a.X = ptr<const void*>(d, "X");
    a.W = ptr<const void*>(d, "W");
    a.bias = ptr<const float*>(d, "bias");
    a.Y = ptr<void*>(d, "Y");
    a.m_ptr = ptr<const int32_t*>(d, "m_ptr");
    a.M = geti(d, "M");
    a.N = geti(d, "N");
    a.K = geti(d, "K");
    a.ldx = geti(d, "ldx");
    a.ldy = geti(d, "ldy");
    a.ldw = geti(d, "ldw");
    a.x_bf16 = geti(d, "x_bf16");
    a.y_bf16 = geti(d, "y_bf16");
    a.act = geti(d, "act");
    a.w_f32 = geti(d, "w_f32", 0);
    return a;
  };
  m.def("gemm", [gemm_args](py::dict d, uintptr_t s) {
    const GemmArgs a = gemm_args(d);
    launch_or_record([a](hipStream_t st) { launch_gemm(a, st); }, s, "gemm");
  });
  m.def("gemv", [gemm_args](py::dict d, uintptr_t s) {
    const GemmArgs a = gemm_args(d);
    launch_or_record([a](hipStream_t st) { launch_gemv(a, st); }, s, "gemv");
  });
  m.def("join", [](py::dict d, uintptr_t s) {
    JoinArgs a{};
    a.A = ptr<const void*>(d, "A");
    a.B = ptr<const void*>(d, "B");
    a.Y = ptr<void*>(d, "Y");
    a.m_ptr = ptr<const int32_t*>(d, "m_ptr");
    a.M = geti(d, "M");
    a.na = geti(d, "na");
    a.nb = geti(d, "nb");
    a.op = geti(d, "op");
    a.lda = geti(d, "lda");
    a.ldb = geti(d, "ldb");
    a.ldy = geti(d, "ldy");
    a.a_bf16 = geti(d, "a_bf16");
    a.b_bf16 = geti(d, "b_bf16");
    a.y_bf16 = geti(d, "y_bf16");
    if (!a.A || !a.B || !a.Y || a.na < 1 || (a.op != 0 && a.op != 1)) throw std::runtime_error("join: args");
    if (a.op == 0 && a.nb != a.na) throw std::runtime_error("join: add needs equal widths");
    if (a.op == 1 && a.nb < 1) throw std::runtime_error("join: concat widths");
    launch_or_record([a](hipStream_t st) { launch_join(a, st); }, s, "join");
  });

  auto head_args = [](const py::dict& d) {
    HeadArgs a{};
    a.X = ptr<const void*>(d, "X");
    a.W1 = ptr<const void*>(d, "W1");
    a.w1_f32 = geti(d, "w1_f32", 0);
    a.b1 = ptr<const float*>(d, "b1");
    a.w2 = ptr<const float*>(d, "w2");
    a.b2 = d.contains("b2") ? d["b2"].cast<float>() : 0.f;
    a.Y = ptr<float*>(d, "Y");
    a.m_ptr = ptr<const int32_t*>(d, "m_ptr");
    a.M = geti(d, "M");
    a.K = geti(d, "K");
    a.N1 = geti(d, "N1");
    a.k_pad = geti(d, "k_pad");
    a.ldx = geti(d, "ldx");
    a.ldy = geti(d, "ldy");
    a.x_bf16 = geti(d, "x_bf16");
    a.act1 = geti(d, "act1");
    a.act2 = geti(d, "act2");
    a.partial = ptr<const float*>(d, "partial");
    a.pbase = ptr<const float*>(d, "pbase");
    a.groups = geti(d, "groups", 1);
    a.p_average = geti(d, "p_average", 0);
    a.p_ntrees = geti(d, "p_ntrees", 1);
    a.trace = ptr<int64_t*>(d, "trace");
    if (d.contains("ens") && !d["ens"].is_none()) {
      a.fuse_ens = 1;
      a.ens = ensemble_args(d["ens"].cast<py::dict>());
      if (!a.ens.hdr || !a.ens.cfg || !a.ens.feat || !a.ens.out) throw std::runtime_error("mlp_head: ensemble args");
    }
    if (a.k_pad % 32 || a.k_pad < a.K) throw std::runtime_error("mlp_head: k_pad must be a multiple of 32 >= K");
    return a;
  };

  m.def("mlp_head", [head_args](py::dict d, uintptr_t s) {
    const HeadArgs a = head_args(d);
    launch_or_record([a](hipStream_t st) { launch_mlp_head(a, st); }, s, "mlp_head");
  });

  m.def("tree_head", [tree_args, head_args](py::dict dt, py::dict dh, uintptr_t s) {
    const TreeArgs a = tree_args(dt);
    const HeadArgs h = head_args(dh);
    const int groups = geti(dt, "groups", 1);
    float* partial = ptr<float*>(dt, "partial");
    unsigned int* cnt = ptr<unsigned int*>(dt, "tile_cnt");
    if (!partial || !cnt || h.partial != partial || h.groups != groups)
      throw std::runtime_error("tree_head: partial slab / tile counters");
    if (!tree_head_supported(a, h, groups)) throw std::runtime_error("tree_head: unsupported tree/head shape");
    launch_or_record([a, h, groups, partial, cnt](hipStream_t st) { launch_tree_head(a, h, groups, partial, cnt, st); },
                     s, "tree_head");
  });

  m.def("ensemble", [](py::dict d, uintptr_t s) {
    const EnsembleArgs a = ensemble_args(d);
    launch_or_record([a](hipStream_t st) { launch_ensemble(a, st); }, s, "ensemble");
  });

  m.def("ltv", [](py::dict d, uintptr_t s) {
    LtvArgs a{};
    a.pf = ptr<const float*>(d, "pf");
    a.ltv_model = ptr<const float*>(d, "ltv_model");
    a.slots = ptr<const int32_t*>(d, "slots");
    a.out = ptr<float*>(d, "out");
    a.B = geti(d, "B");
    launch_or_record([a](hipStream_t st) { launch_ltv(a, st); }, s, "ltv");
  });
  m.def("ltv_assemble", [](py::dict d, uintptr_t s) {
    LtvAssembleArgs a{};
    a.slots = ptr<const int32_t*>(d, "slots");
    a.pf_tab = ptr<const float*>(d, "pf_tab");
    a.ext_tab = ptr<const float*>(d, "ext_tab");
    a.ext_w = geti(d, "ext_w");
    a.X = ptr<float*>(d, "X");
    a.x_w = geti(d, "x_w");
    a.m_ptr = ptr<const int32_t*>(d, "m_ptr");
    a.n_rows = geti(d, "n_rows");
    if (!a.slots || !a.pf_tab || !a.X || a.x_w < 25) throw std::runtime_error("ltv_assemble: bad args");
    launch_or_record([a](hipStream_t st) { launch_ltv_assemble(a, st); }, s, "ltv_assemble");
  });
  m.def("gru", [](py::dict d, uintptr_t s) {
    GruArgs a{};
    a.n_layers = geti(d, "n_layers");
    if (a.n_layers < 1 || a.n_layers > 2) throw std::runtime_error("gru: 1 or 2 layers");
    for (int l = 0; l < a.n_layers; ++l) {
      const std::string p = "l" + std::to_string(l) + "_";
      a.layer[l].W = ptr<const uint16_t*>(d, (p + "W").c_str());
      a.layer[l].R = ptr<const uint16_t*>(d, (p + "R").c_str());
      a.layer[l].bias = ptr<const float*>(d, (p + "bias").c_str());
      a.layer[l].kx_pad = geti(d, (p + "kx_pad").c_str());
      a.layer[l].lbr = geti(d, (p + "lbr").c_str());
      a.layer[l].W_lo = ptr<const uint16_t*>(d, (p + "Wlo").c_str());
      a.layer[l].R_lo = ptr<const uint16_t*>(d, (p + "Rlo").c_str());
      if (!a.layer[l].W || !a.layer[l].R || !a.layer[l].bias) throw std::runtime_error("gru: missing layer weights");
    }
    a.H = geti(d, "H");
    a.T = geti(d, "T");
    a.I = geti(d, "I");
    a.mode = geti(d, "mode");
    a.X = ptr<const float*>(d, "X");
    a.x_rows = geti(d, "x_rows");
    a.ev = ptr<const uint16_t*>(d, "ev");
    a.rt = ptr<const AcctRT*>(d, "rt");
    a.slots = ptr<const int32_t*>(d, "slots");
    a.ev_ring = geti(d, "ev_ring");
    a.m_ptr = ptr<const int32_t*>(d, "m_ptr");
    a.n_rows = geti(d, "n_rows");
    a.yh = ptr<float*>(d, "yh");
    a.head_w = ptr<const float*>(d, "head_w");
    a.head_b = d.contains("head_b") ? d["head_b"].cast<float>() : 0.f;
    a.head_act = geti(d, "head_act");
    a.out = ptr<float*>(d, "out");
    a.tile_rows = geti(d, "tile_rows");
    a.waves = geti(d, "waves");
    a.pipeline = geti(d, "pipeline", 1);
    a.ws = geti(d, "ws");
    a.ws_clusters = geti(d, "ws_clusters");
    a.ws_sync = ptr<int32_t*>(d, "ws_sync");
    a.ws_x = ptr<uint16_t*>(d, "ws_x");
    a.ws_part = ptr<float*>(d, "ws_part");
    a.ws_err = ptr<int32_t*>(d, "ws_err");
    a.ws_trace = ptr<int64_t*>(d, "ws_trace");
    a.split = geti(d, "split");
    a.reverse = geti(d, "reverse", 0);
    if (a.split) {
      for (int l = 0; l < a.n_layers; ++l)
        if (!a.layer[l].W_lo || !a.layer[l].R_lo) throw std::runtime_error("gru: split mode needs residual weights");
    }
    if (a.tile_rows != 0 && a.tile_rows != 16 && a.tile_rows != 32) throw std::runtime_error("gru: tile_rows 16|32");
    if (a.H != 64 && a.H != 128 && a.H != 256) throw std::runtime_error("gru: H must be 64, 128 or 256");
    if (a.layer[0].kx_pad != 32 && a.layer[0].kx_pad != 64) throw std::runtime_error("gru: input dim must pad to 32 or 64");
    if (a.n_layers == 2 && a.layer[1].kx_pad != a.H) throw std::runtime_error("gru: layer 2 input must be H");
    if (a.I % 8 != 0 || a.I > a.layer[0].kx_pad) throw std::runtime_error("gru: I must be a multiple of 8 <= kx_pad");
    if (a.mode == 1 && (!a.ev || !a.rt || !a.slots || a.ev_ring < a.T)) throw std::runtime_error("gru: event-ring input");
    if (a.mode == 0 && (!a.X || a.x_rows < a.n_rows)) throw std::runtime_error("gru: dense input");
    if (a.head_w && !a.out) throw std::runtime_error("gru: head needs out");
    if (recording()) throw std::runtime_error("gru: not recordable (host-side scratch resets); use graphs");
    launch_gru(a, stream_of(s));
    check("gru");
  });
  m.def("gru_ws_clusters", [](int n_rows) { return gru_ws_clusters(n_rows); });

  m.def("mlp_chain", [](py::dict d, uintptr_t s) {
    MlpChainArgs a{};
    a.X = ptr<const float*>(d, "X");
    a.ldx = geti(d, "ldx");
    a.slots = ptr<const int32_t*>(d, "slots");
    a.pf_tab = ptr<const float*>(d, "pf_tab");
    a.ext_tab = ptr<const float*>(d, "ext_tab");
    a.ext_w = geti(d, "ext_w");
    a.in_w = geti(d, "in_w");
    a.in_live = geti(d, "in_live");
    a.m_ptr = ptr<const int32_t*>(d, "m_ptr");
    a.n_rows = geti(d, "n_rows");
    a.n_layers = geti(d, "n_layers");
    if (a.n_layers < 1 || a.n_layers > MC_MAX_LAYERS) throw std::runtime_error("mlp_chain: 1..8 layers");
    for (int l = 0; l < a.n_layers; ++l) {
      const std::string p = "l" + std::to_string(l) + "_";
      a.W[l] = ptr<const uint16_t*>(d, (p + "W").c_str());
      a.bias[l] = ptr<const float*>(d, (p + "b").c_str());
      a.N[l] = geti(d, (p + "N").c_str());
      a.K[l] = geti(d, (p + "K").c_str());
      a.act[l] = geti(d, (p + "act").c_str());
      a.W_lo[l] = ptr<const uint16_t*>(d, (p + "Wlo").c_str());
      if (!a.W[l]) throw std::runtime_error("mlp_chain: missing weights");
      if (a.N[l] < 64 || a.N[l] > 512 || a.N[l] % 64) throw std::runtime_error("mlp_chain: N must be 64..512, % 64");
      if (a.K[l] < 64 || a.K[l] > 512 || a.K[l] % 64) throw std::runtime_error("mlp_chain: K must be 64..512, % 64");
      if (l > 0 && a.K[l] != a.N[l - 1]) throw std::runtime_error("mlp_chain: K[l] != N[l-1]");
    }
    if (a.in_w != a.K[0] || a.in_live > a.in_w || a.in_live < 1) throw std::runtime_error("mlp_chain: input width");
    a.w2 = ptr<const float*>(d, "w2");
    a.b2 = d.contains("b2") ? d["b2"].cast<float>() : 0.f;
    a.act2 = geti(d, "act2");
    a.ml = ptr<float*>(d, "ml");
    a.ltv_out = ptr<float*>(d, "ltv_out");
    a.rows_per_block = geti(d, "rows_per_block", 32);
    a.waves = geti(d, "waves", 4);
    if (a.rows_per_block != 16 && a.rows_per_block != 32 && a.rows_per_block != 64)
      throw std::runtime_error("mlp_chain: 16, 32 or 64 rows per block");
    if (a.waves != 4 && a.waves != 8) throw std::runtime_error("mlp_chain: 4 or 8 waves");
    for (int l = 0; l < a.n_layers; ++l)
      if (a.N[l] % (16 * a.waves)) throw std::runtime_error("mlp_chain: N must be a multiple of 16 x waves");
    a.split = geti(d, "split", 0);
    if (a.split) {
      for (int l = 0; l < a.n_layers; ++l)
        if (!a.W_lo[l]) throw std::runtime_error("mlp_chain: split mode needs every layer's residual weights");
      if (a.rows_per_block != 32 && !(a.rows_per_block == 64 && a.waves == 8))
        throw std::runtime_error("mlp_chain: split mode runs 32 rows per block (64 with 8 waves)");
    }
    if (!a.w2) throw std::runtime_error("mlp_chain: head weights required");
    if (!a.slots && !a.X) throw std::runtime_error("mlp_chain: input");
    if (a.slots && !a.pf_tab) throw std::runtime_error("mlp_chain: LTV gather needs the profile table");
    if (a.ltv_out && !a.slots) throw std::runtime_error("mlp_chain: the K9 epilogue needs slots");
    launch_or_record([a](hipStream_t st) { launch_mlp_chain(a, st); }, s, "mlp_chain");
  });
}
