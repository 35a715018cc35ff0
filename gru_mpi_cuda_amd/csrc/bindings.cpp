// Thin pybind11 layer over the native engine.  No torch headers: device memory is passed as
// integer addresses (tensor.data_ptr()) and streams as integer handles
// (torch.cuda.current_stream().cuda_stream), so this TU compiles in seconds and the
// extension binds to whichever libamdhip64 the process already loaded (torch's).
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include "engine/trainer.h"
#include "engine/generator.h"
#include "comm/rccl_comm.h"
#include "comm/bootstrap.h"
#include "data/name_loader.h"

namespace py = pybind11;
using namespace gk;

static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
template <class T> static T* Pp(uintptr_t p) { return reinterpret_cast<T*>(p); }

template <class T>
static T get(const py::dict& d, const char* k, T dflt) {
  if (!d.contains(k)) return dflt;
  return d[k].cast<T>();
}
#define GP(T, d, k) reinterpret_cast<T*>(get<uintptr_t>(d, k, 0))

PYBIND11_MODULE(_C, m) {
  m.doc() = "gru_mpi_cuda_amd native engine (HIP/CDNA4 kernels, hipGraph executor, RCCL comm)";

  m.def("set_rank", [](int r) { global_rank() = r; });

  py::class_<NameLoader>(m, "NameLoader")
      .def(py::init([](py::dict d) {
        LoaderCfg c;
        c.B = get<int>(d, "B", 256); c.T = get<int>(d, "T", 32);
        c.sos = get<int>(d, "sos", 0); c.eos = get<int>(d, "eos", 0); c.max_len = get<int>(d, "max_len", 10);
        c.seed = get<uint64_t>(d, "seed", 0); c.prefetch = get<int>(d, "prefetch", 4);
        c.path = get<std::string>(d, "path", "");
        return new NameLoader(c);
      }))
      .def("next", [](NameLoader& L, int B, int T) {
        py::array_t<int32_t> x({B, T}), y({B, T});
        int32_t* px = x.mutable_data();
        int32_t* py_ = y.mutable_data();
        {
          py::gil_scoped_release nogil;   // the producer thread may still be filling the batch
          L.next(px, py_);
        }
        return py::make_tuple(x, y);
      })
      .def("batches", &NameLoader::batches)
      .def("epoch", &NameLoader::epoch)
      .def("names_in_file", &NameLoader::names_in_file);
  m.def("device_info", []() {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    hipDeviceProp_t p;
    HIP_CHECK(hipGetDeviceProperties(&p, dev));
    py::dict d;
    d["name"] = std::string(p.name);
    d["arch"] = std::string(p.gcnArchName);
    d["cus"] = p.multiProcessorCount;
    d["lds_per_cu"] = (long)p.maxSharedMemoryPerMultiProcessor;
    d["hbm_bytes"] = (long)p.totalGlobalMem;
    return d;
  });
  m.def("device_synchronize", []() { HIP_CHECK(hipDeviceSynchronize()); });

  py::class_<Trainer>(m, "Trainer")
      .def(py::init([](py::dict dims, py::dict opt, uintptr_t params, uintptr_t grads, uintptr_t mm, uintptr_t vv,
                       long nflat, std::map<std::string, long> offsets) {
        Dims d;
        d.V = get<int>(dims, "V", 256); d.E = get<int>(dims, "E", 512); d.H = get<int>(dims, "H", 512);
        d.L = get<int>(dims, "L", 1); d.B = get<int>(dims, "B", 256); d.T = get<int>(dims, "T", 32);
        d.chunks = get<int>(dims, "chunks", 4); d.overlap = get<int>(dims, "overlap", 1);
        OptCfg o;
        o.lr = get<float>(opt, "lr", 1e-3f); o.b1 = get<float>(opt, "beta1", 0.9f); o.b2 = get<float>(opt, "beta2", 0.999f);
        o.eps = get<float>(opt, "eps", 1e-8f); o.wd = get<float>(opt, "weight_decay", 0.f);
        o.clip = get<float>(opt, "clip_norm", 0.f); o.sgd = get<int>(opt, "sgd", 0);
        o.sched = get<int>(opt, "lr_sched", 0); o.warmup = get<int>(opt, "warmup_steps", 0);
        o.total = get<int>(opt, "total_steps", 0); o.lr_min = get<float>(opt, "lr_min", 0.f);
        o.keep_grads = get<int>(opt, "keep_grads", 1);
        return new Trainer(d, o, Pp<float>(params), Pp<float>(grads), Pp<float>(mm), Pp<float>(vv), nflat, offsets);
      }))
      .def("refresh_weights", [](Trainer& t, uintptr_t s) { t.refresh_weights(S(s)); })
      .def("set_batch", [](Trainer& t, py::array_t<int, py::array::c_style | py::array::forcecast> x,
                           py::array_t<int, py::array::c_style | py::array::forcecast> y, uintptr_t s) {
        if (x.ndim() != 2 || y.ndim() != 2 || x.shape(0) != y.shape(0) || x.shape(1) != y.shape(1))
          throw std::runtime_error("set_batch: x and y must both be [B, T]");
        t.set_batch(x.data(), y.data(), (int)x.shape(0), S(s));
      })
      .def("set_batch_device", [](Trainer& t, uintptr_t x, uintptr_t y, int B, uintptr_t s) {
        t.set_batch_device(Pp<const int>(x), Pp<const int>(y), B, S(s));
      })
      .def("set_comm", [](Trainer& t, RcclComm* c, std::vector<std::pair<long, long>> buckets, long min_bucket) {
        t.set_comm(c, buckets, min_bucket);
      }, py::arg("comm"), py::arg("buckets"), py::arg("min_bucket_floats") = 2L << 20, py::keep_alive<1, 2>())
      .def("allreduce_log", &Trainer::allreduce_log)
      .def("step", [](Trainer& t, uintptr_t s) { t.step(S(s)); })
      .def("set_graph_steps", &Trainer::set_graph_steps)
      .def("graph_steps", &Trainer::graph_steps)
      .def("set_batches", [](Trainer& t, py::array_t<int, py::array::c_style | py::array::forcecast> x,
                             py::array_t<int, py::array::c_style | py::array::forcecast> y) {
        if (x.ndim() != 3 || y.ndim() != 3 || x.shape(0) != y.shape(0) || x.shape(1) != y.shape(1) ||
            x.shape(2) != y.shape(2))
          throw std::runtime_error("set_batches: x and y must both be [G, B, T]");
        t.set_batches(x.data(), y.data(), (int)x.shape(1), (int)x.shape(0));
      })
      .def("step_group", [](Trainer& t, uintptr_t s) { t.step_group(S(s)); })
      .def("forward_backward", [](Trainer& t, uintptr_t s) { t.forward_backward(S(s)); })
      .def("optimizer_step", [](Trainer& t, uintptr_t s) { t.optimizer_step(S(s)); })
      .def("read_loss", &Trainer::read_loss)
      .def("read_grad_norm", &Trainer::read_grad_norm)
      .def("get_step", &Trainer::get_step)
      .def("set_step", &Trainer::set_step)
      .def("set_lr", &Trainer::set_lr)
      .def("set_use_graph", &Trainer::set_use_graph)
      .def("set_carry", &Trainer::set_carry)
      .def("carry", &Trainer::carry)
      .def("reset_hidden", [](Trainer& t, uintptr_t s) { t.reset_hidden(S(s)); })
      .def("padded_batch", &Trainer::padded_batch)
      .def("workspace_bytes", &Trainer::workspace_bytes)
      .def("plan", &Trainer::plan)
      .def("uses_persistent", &Trainer::uses_persistent)
      .def("read_error", &Trainer::read_error)
      .def("enable_watchdog", &Trainer::enable_watchdog)
      .def("set_shard_optim", &Trainer::set_shard_optim)
      .def("set_dp_pipeline", &Trainer::set_dp_pipeline)
      .def("dp_pipeline", &Trainer::dp_pipeline)
      .def("dp_tail_recorded", &Trainer::dp_tail_recorded)
      .def("shard_optim", &Trainer::shard_optim)
      .def("shard_mode", &Trainer::shard_mode)
      .def("gather_params", [](Trainer& t, uintptr_t s) { t.gather_params(S(s)); })
      .def("shard_chunk", &Trainer::shard_chunk)
      .def("gather_opt_state", [](Trainer& t, uintptr_t s) { t.gather_opt_state(S(s)); })
      .def("inject_error", &Trainer::inject_error)
      .def("watchdog_status", &Trainer::watchdog_status)
      .def("watchdog_message", &Trainer::watchdog_message)
      .def("buffer", &Trainer::buffer);

  py::class_<Generator>(m, "Generator")
      .def(py::init([](py::dict dims, uintptr_t params, std::map<std::string, long> offsets) {
        GenDims d;
        d.V = get<int>(dims, "V", 256); d.E = get<int>(dims, "E", 512); d.H = get<int>(dims, "H", 1024);
        d.L = get<int>(dims, "L", 2); d.max_len = get<int>(dims, "max_len", 10); d.sos = get<int>(dims, "sos", 0);
        d.eos = get<int>(dims, "eos", 0); d.max_batch = get<int>(dims, "max_batch", 4096);
        d.fp32 = get<int>(dims, "fp32", 0);
        return new Generator(d, Pp<const float>(params), offsets);
      }))
      .def("refresh_weights", [](Generator& g, uintptr_t s) { g.refresh_weights(S(s)); })
      .def("generate", [](Generator& g, uintptr_t rf, int N, uintptr_t out, uintptr_t s) {
        g.generate(Pp<const float>(rf), N, Pp<unsigned char>(out), S(s));
      })
      .def("set_use_graph", &Generator::set_use_graph)
      .def("read_error", &Generator::read_error)
      .def("set_probe", [](Generator& g, uintptr_t p) { g.set_probe(Pp<float>(p)); })
      .def("set_persist", &Generator::set_persist)
      .def("set_persist_max", &Generator::set_persist_max)
      .def("set_persist_dbg", [](Generator& g, uintptr_t p) { g.set_persist_dbg(reinterpret_cast<unsigned long long*>(p)); })
      .def("uses_persist", &Generator::uses_persist)
      .def("set_global_names", &Generator::set_global_names)
      .def("inject_persist_error", &Generator::inject_persist_error)
      .def("dump_graph", &Generator::dump_graph);

  // ---------------------------------------------------------------- raw kernels (tests, bench)
  m.def("gemm_f32", [](py::dict d, uintptr_t s) {   // fp32 MFMA GEMM of the fp32 generation path
    GemmF32Args a;
    a.A = GP(const float, d, "A"); a.lda = get<int>(d, "lda", 0);
    a.B = GP(const float, d, "B"); a.ldb = get<int>(d, "ldb", 0);
    a.C = GP(float, d, "C"); a.ldc = get<int>(d, "ldc", 0);
    a.bias = GP(const float, d, "bias");
    a.M = get<int>(d, "M", 0); a.N = get<int>(d, "N", 0); a.K = get<int>(d, "K", 0);
    a.splits = get<int>(d, "splits", 1); a.slab = get<long>(d, "slab", 0);
    gemm_f32_nt(a, S(s));
  });
  m.def("gemm_nt", [](py::dict d, uintptr_t s) {
    GemmArgs a;
    a.A = GP(const u16, d, "A"); a.lda = get<int>(d, "lda", 0);
    a.onehot_ids = GP(const int, d, "onehot_ids");
    a.B2 = GP(const u16, d, "B2"); a.b2_row = get<int>(d, "b2_row", 0);
    a.B = GP(const u16, d, "B"); a.ldb = get<int>(d, "ldb", 0);
    a.C = GP(float, d, "C"); a.ldc = get<int>(d, "ldc", 0);
    a.bias = GP(const float, d, "bias"); a.rowsumA = GP(float, d, "rowsumA");
    a.M = get<int>(d, "M", 0); a.N = get<int>(d, "N", 0); a.K = get<int>(d, "K", 0);
    a.splits = get<int>(d, "splits", 1); a.accumulate = get<int>(d, "accumulate", 0);
    a.algo = get<int>(d, "algo", 0);
    if (a.M % 64 || a.N % 64 || (a.K / a.splits) % 32 || a.K % a.splits)
      throw std::runtime_error("gemm_nt: M, N must be multiples of 64 and K/splits a multiple of 32");
    gemm_nt(a, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("cast_multi", [](py::list jobs, uintptr_t s) {
    CastJobs j;
    if (jobs.size() > 24) throw std::runtime_error("cast_multi: at most 24 jobs");
    for (auto h : jobs) {
      py::dict d = h.cast<py::dict>();
      j.add(GP(const float, d, "src"), get<int>(d, "R", 0), get<int>(d, "C", 0), GP(u16, d, "dst"),
            GP(u16, d, "dstT"), GP(u16, d, "dstF"), GP(u16, d, "dstTF"));
    }
    cast_multi(j, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("reduce_slabs_cast", [](py::dict d, uintptr_t s) {   // one slab-sum + cast job
    SlabJobs j;
    j.add_cast(GP(const float, d, "src"), get<int>(d, "splits", 1), get<int>(d, "R", 0), get<int>(d, "C", 0),
               GP(float, d, "dst"), GP(u16, d, "bf"), GP(u16, d, "bfT"));
    reduce_slabs_multi(j, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("fwd_step", [](py::dict d, uintptr_t s) {
    FwdStepArgs a;
    a.hprev_bf = GP(const u16, d, "hprev_bf"); a.hprev_f = GP(const float, d, "hprev_f");
    a.Whh = GP(const u16, d, "Whh"); a.bhh = GP(const float, d, "bhh");
    a.P = GP(const float, d, "P"); a.ids = GP(const int, d, "ids"); a.Gi = GP(const float, d, "Gi");
    a.x_bf = GP(const u16, d, "x_bf"); a.Wih = GP(const u16, d, "Wih"); a.bih = GP(const float, d, "bih");
    a.Kin = get<int>(d, "Kin", 0);
    a.h_f = GP(float, d, "h_f"); a.h_bf = GP(u16, d, "h_bf"); a.hT = GP(u16, d, "hT");
    a.ldT = get<int>(d, "ldT", 0); a.colT = get<int>(d, "colT", 0);
    a.sr = GP(float, d, "sr"); a.sz = GP(float, d, "sz"); a.sn = GP(float, d, "sn"); a.sghn = GP(float, d, "sghn");
    a.Bp = get<int>(d, "Bp", 0); a.H = get<int>(d, "H", 0); a.algo = get<int>(d, "algo", 0);
    if (a.Bp % 32 || a.H % 64) throw std::runtime_error("fwd_step: Bp % 32 and H % 64 required");
    gru_fwd_step(a, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("bwd_step", [](py::dict d, uintptr_t s) {
    BwdStepArgs a;
    a.dgh_next = GP(const u16, d, "dgh_next"); a.WhhT = GP(const u16, d, "WhhT");
    a.carry_in = GP(const float, d, "carry_in"); a.dy = GP(const float, d, "dy");
    a.r = GP(const float, d, "r"); a.z = GP(const float, d, "z"); a.n = GP(const float, d, "n");
    a.ghn = GP(const float, d, "ghn"); a.hprev = GP(const float, d, "hprev");
    a.carry_out = GP(float, d, "carry_out"); a.dgh = GP(u16, d, "dgh"); a.dghT = GP(u16, d, "dghT");
    a.dgiT = GP(u16, d, "dgiT"); a.dgi = GP(u16, d, "dgi");
    a.ldT = get<int>(d, "ldT", 0); a.colT = get<int>(d, "colT", 0);
    a.Bp = get<int>(d, "Bp", 0); a.H = get<int>(d, "H", 0); a.algo = get<int>(d, "algo", 0);
    a.sk_part = GP(float, d, "sk_part"); a.sk_part_floats = get<long>(d, "sk_part_floats", 0);
    a.sk_cnt = GP(unsigned, d, "sk_cnt"); a.sk_cnt_words = get<long>(d, "sk_cnt_words", 0);
    a.err = GP(unsigned, d, "err");
    a.dgiT_n_only = get<int>(d, "dgiT_n_only", 0);
    if (a.Bp % 32 || a.H % 64) throw std::runtime_error("bwd_step: Bp % 32 and H % 64 required");
    gru_bwd_step(a, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("spin_delay", [](int us, uintptr_t s) { spin_delay(us, S(s)); HIP_LAUNCH_CHECK(); });
  // tests: copy an internal device buffer (Trainer::buffer) into a caller tensor
  m.def("copy_d2d", [](uintptr_t dst, uintptr_t src, size_t bytes) {
    HIP_CHECK(hipMemcpy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), bytes, hipMemcpyDeviceToDevice));
  });
  m.def("graph_node_probe_detail", &graph_node_probe_detail);
  m.def("graph_node_probe", &graph_node_probe);
  m.def("block_cus", [](int nblocks, int us, uintptr_t s) { block_cus(nblocks, us, S(s)); });
  m.def("xcc_census", [](uintptr_t out, int nblocks, int threads, uintptr_t s) {
    xcc_census(Pp<unsigned>(out), nblocks, threads, S(s)); HIP_LAUNCH_CHECK(); });
  m.def("fwd_seq_supported", &gru_fwd_seq_supported);
  m.def("bwd_step_sk_splits", &gru_bwd_step_sk_splits);
  m.def("step_lds_variants", []() {
    const StepLdsVariants& v = step_lds_variants();
    py::dict d;
    d["fwd64"] = v.fwd64; d["bwd_sk_min_h"] = v.bwd_sk_min_h; d["dwfc_group"] = v.dwfc_group;
    d["bwd_big"] = v.bwd_big; d["bwd16"] = v.bwd16; d["bwd_xring"] = v.bwd_xring; d["fwd_xring"] = v.fwd_xring; d["fwd_fc"] = v.fwd_fc; d["fc_flash"] = v.fc_flash; d["save16"] = v.save16; d["big_dy"] = v.big_dy; d["ld_pad"] = v.ld_pad;
    return d;
  });
  m.def("set_step_lds_variants", [](py::dict d) {
    StepLdsVariants& v = step_lds_variants();
    for (auto kv : d) {
      const std::string k = py::str(kv.first);
      const int x = kv.second.cast<int>();
      if (k == "fwd64") v.fwd64 = x;
      else if (k == "bwd_sk_min_h") v.bwd_sk_min_h = x;
      else if (k == "dwfc_group") v.dwfc_group = x;
      else if (k == "bwd_big") v.bwd_big = x;
      else if (k == "bwd16") v.bwd16 = x;
      else if (k == "bwd_xring") v.bwd_xring = x;
      else if (k == "fwd_xring") v.fwd_xring = x;
      else if (k == "fwd_fc") v.fwd_fc = x;
      else if (k == "fc_flash") v.fc_flash = x;
      else if (k == "big_dy") v.big_dy = x;
      else if (k == "ld_pad") v.ld_pad = x;
      else if (k == "save16") v.save16 = x;
      else throw std::runtime_error("set_step_lds_variants: unknown field " + k);
    }
  });
  m.def("gemm_variants", []() {
    const GemmVariants& v = gemm_variants();
    py::dict d;
    d["mfma"] = v.mfma; d["phased"] = v.phased; d["sched"] = v.sched; d["groupm"] = v.groupm; d["onehot"] = v.onehot;
    return d;
  });
  m.def("set_gemm_variants", [](py::dict d) {
    GemmVariants& v = gemm_variants();
    for (auto kv : d) {
      const std::string k = py::str(kv.first);
      const int x = kv.second.cast<int>();
      if (k == "mfma") v.mfma = x;
      else if (k == "phased") v.phased = x;
      else if (k == "sched") v.sched = x;
      else if (k == "groupm") v.groupm = x;
      else if (k == "onehot") v.onehot = x;
      else throw std::runtime_error("set_gemm_variants: unknown field " + k);
    }
  });
  m.def("bwd_seq_supported", &gru_bwd_seq_supported);
  m.def("fwd_seq2", [](py::dict lo, py::dict hi, uintptr_t Wih, uintptr_t bih, uintptr_t s) {
    auto parse = [](py::dict d) {
      SeqFwdArgs a;
      a.HSb = GP(u16, d, "HSb"); a.HSf = GP(float, d, "HSf"); a.HT = GP(u16, d, "HT"); a.ldT = get<int>(d, "ldT", 0);
      a.HF = GP(u16, d, "HF"); a.xch = GP(u16, d, "xch");
      a.sr = GP(float, d, "sr"); a.sz = GP(float, d, "sz"); a.sn = GP(float, d, "sn"); a.sghn = GP(float, d, "sghn");
      a.Whh = GP(const u16, d, "Whh"); a.bhh = GP(const float, d, "bhh");
      a.P = GP(const float, d, "P"); a.ids = GP(const int, d, "ids"); a.Gi = GP(const float, d, "Gi");
      a.h0 = GP(const float, d, "h0");
      a.cnt = GP(unsigned, d, "cnt"); a.err = GP(unsigned, d, "err");
      a.dbg = GP(unsigned long long, d, "dbg"); a.allow_local = get<int>(d, "allow_local", 1);
      a.xring = get<int>(d, "xring", 0);
      a.T = get<int>(d, "T", 0); a.Bp = get<int>(d, "Bp", 0); a.H = get<int>(d, "H", 0);
      if (!a.xch || !a.cnt || !a.HSb || !a.HSf || !a.Whh || !a.bhh) throw std::runtime_error("fwd_seq2: HSb/HSf/xch/cnt/Whh/bhh required");
      return a;
    };
    SeqFwd2Args a;
    a.lo = parse(lo); a.hi = parse(hi);
    a.Wih = reinterpret_cast<const u16*>(Wih); a.bih = reinterpret_cast<const float*>(bih);
    if (!a.lo.ids == !a.lo.Gi) throw std::runtime_error("fwd_seq2: lo needs exactly one of P+ids / Gi");
    if (!gru_fwd_seq2_supported(a.lo.H, a.lo.Bp)) throw std::runtime_error("fwd_seq2: shape not supported");
    gru_fwd_seq2(a, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("fwd_seq2_supported", &gru_fwd_seq2_supported);
  m.def("fwd_seq_fc_supported", &gru_fwd_seq_fc_supported);
  m.def("fwd_seq_fc", [](py::dict d, py::dict fd, uintptr_t s) {
    SeqFwdArgs a;
    a.HSb = GP(u16, d, "HSb"); a.HSf = GP(float, d, "HSf"); a.HT = GP(u16, d, "HT"); a.ldT = get<int>(d, "ldT", 0);
    a.HF = GP(u16, d, "HF"); a.xch = GP(u16, d, "xch");
    a.sr = GP(float, d, "sr"); a.sz = GP(float, d, "sz"); a.sn = GP(float, d, "sn"); a.sghn = GP(float, d, "sghn");
    a.Whh = GP(const u16, d, "Whh"); a.bhh = GP(const float, d, "bhh");
    a.P = GP(const float, d, "P"); a.ids = GP(const int, d, "ids"); a.Gi = GP(const float, d, "Gi");
    a.h0 = GP(const float, d, "h0");
    a.cnt = GP(unsigned, d, "cnt"); a.err = GP(unsigned, d, "err");
    a.dbg = GP(unsigned long long, d, "dbg"); a.allow_local = get<int>(d, "allow_local", 1);
    a.xring = get<int>(d, "xring", 0);
    a.T = get<int>(d, "T", 0); a.Bp = get<int>(d, "Bp", 0); a.H = get<int>(d, "H", 0);
    SeqFcArgs f;
    f.Wf = GP(const u16, fd, "Wf"); f.WTf = GP(const u16, fd, "WTf"); f.b = GP(const float, fd, "b");
    f.labels = GP(const int, fd, "labels"); f.inv_count = GP(const float, fd, "inv_count");
    f.dy = GP(float, fd, "dy"); f.dlF = GP(u16, fd, "dlF"); f.loss_part = GP(float, fd, "loss_part");
    f.dW = GP(float, fd, "dW"); f.db = GP(float, fd, "db"); f.V = get<int>(fd, "V", 0);
    f.probe = get<int>(fd, "probe", 0);
    if (!a.xch || !a.cnt || !a.HSb || !a.HSf || !a.Whh || !a.bhh) throw std::runtime_error("fwd_seq_fc: HSb/HSf/xch/cnt/Whh/bhh required");
    if (!gru_fwd_seq_fc_supported(a.H, a.Bp, f.V)) throw std::runtime_error("fwd_seq_fc: shape not supported");
    gru_fwd_seq_fc(a, f, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("fwd_seq", [](py::dict d, uintptr_t s) {
    SeqFwdArgs a;
    a.HSb = GP(u16, d, "HSb"); a.HSf = GP(float, d, "HSf"); a.HT = GP(u16, d, "HT"); a.ldT = get<int>(d, "ldT", 0);
    a.HF = GP(u16, d, "HF");
    a.xch = GP(u16, d, "xch");
    if (!a.xch) throw std::runtime_error("fwd_seq: exchange buffer xch [T][Bp][H] bf16 required");
    a.sr = GP(float, d, "sr"); a.sz = GP(float, d, "sz"); a.sn = GP(float, d, "sn"); a.sghn = GP(float, d, "sghn");
    a.Whh = GP(const u16, d, "Whh"); a.bhh = GP(const float, d, "bhh");
    a.P = GP(const float, d, "P"); a.ids = GP(const int, d, "ids"); a.Gi = GP(const float, d, "Gi");
    a.h0 = GP(const float, d, "h0");
    a.cnt = GP(unsigned, d, "cnt"); a.err = GP(unsigned, d, "err");
    a.dbg = GP(unsigned long long, d, "dbg"); a.allow_local = get<int>(d, "allow_local", 1);
    a.xring = get<int>(d, "xring", 0);
    a.T = get<int>(d, "T", 0); a.Bp = get<int>(d, "Bp", 0); a.H = get<int>(d, "H", 0);
    if (!gru_fwd_seq_supported(a.H, a.Bp)) throw std::runtime_error("fwd_seq: shape not supported");
    gru_fwd_seq(a, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("bwd_seq_big_supported", &gru_bwd_seq_big_supported);
  m.def("bwd_seq", [](py::dict d, uintptr_t s) {
    SeqBwdArgs a;
    a.dy = GP(const float, d, "dy");
    a.sr = GP(const float, d, "sr"); a.sz = GP(const float, d, "sz"); a.sn = GP(const float, d, "sn");
    a.sghn = GP(const float, d, "sghn"); a.HSf = GP(const float, d, "HSf");
    a.HT = GP(const u16, d, "HT"); a.ldT = get<int>(d, "ldT", 0); a.WhhT = GP(const u16, d, "WhhT");
    a.HF = GP(const u16, d, "HF");
    a.xbuf = GP(u16, d, "xbuf"); a.dghT = GP(u16, d, "dghT"); a.dgiT = GP(u16, d, "dgiT");
    a.ldG = get<int>(d, "ldG", 0); a.dgi = GP(u16, d, "dgi");
    a.dWhh_part = GP(float, d, "dWhh_part"); a.dbhh_part = GP(float, d, "dbhh_part");
    a.dbih_part = GP(float, d, "dbih_part"); a.ids = GP(const int, d, "ids");
    a.dP_part = GP(float, d, "dP_part"); a.V = get<int>(d, "V", 0);
    a.cnt = GP(unsigned, d, "cnt"); a.err = GP(unsigned, d, "err"); a.dbg = GP(unsigned long long, d, "dbg");
    a.allow_local = get<int>(d, "allow_local", 1); a.xring = get<int>(d, "xring", 0);
    a.T = get<int>(d, "T", 0); a.Bp = get<int>(d, "Bp", 0); a.H = get<int>(d, "H", 0);
    // "unchecked": skip the co-residency query and go straight to the dispatch table (tests its
    // unmatched-variant error without launching anything)
    if (get<int>(d, "rows16", 0)) {   // the 16-row-block backward (gru_seq16.hip)
      if (!gru_bwd_seq16_supported(a.H, a.Bp, a.dP_part != nullptr)) throw std::runtime_error("bwd_seq(rows16): shape not supported");
      gru_bwd_seq16(a, S(s));
      HIP_LAUNCH_CHECK();
      return;
    }
    if (!get<int>(d, "unchecked", 0) &&
        !gru_bwd_seq_supported(a.H, a.Bp, a.dWhh_part != nullptr, a.dP_part != nullptr))
      throw std::runtime_error("bwd_seq: shape not supported");
    gru_bwd_seq(a, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("fc_xent", [](py::dict d, uintptr_t s) {
    FcXentArgs a;
    a.X = GP(const u16, d, "X"); a.W = GP(const u16, d, "W"); a.b = GP(const float, d, "b");
    a.labels = GP(const int, d, "labels"); a.inv_count = GP(const float, d, "inv_count");
    a.dl = GP(u16, d, "dl"); a.dlT = GP(u16, d, "dlT"); a.loss_part = GP(float, d, "loss_part");
    a.M = get<int>(d, "M", 0); a.H = get<int>(d, "H", 0); a.V = get<int>(d, "V", 0);
    a.ldT = get<int>(d, "ldT", 0); a.colT = get<int>(d, "colT", 0);
    a.WT = GP(const u16, d, "WT"); a.dy = GP(float, d, "dy");
    a.dbg = GP(unsigned long long, d, "dbg");
    a.Wf = GP(const u16, d, "Wf"); a.WTf = GP(const u16, d, "WTf");
    if (a.M % 32 || a.V % 64 || a.V > 512 || a.H % 32 || a.ldT % 8 || a.colT % 8)
      throw std::runtime_error("fc_xent: bad shape");
    fc_xent(a, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("fc_sample", [](py::dict d, uintptr_t s) {
    FcSampleArgs a;
    a.X = GP(const u16, d, "X"); a.W = GP(const u16, d, "W"); a.b = GP(const float, d, "b");
    a.Wf = GP(const u16, d, "Wf");
    a.rf = GP(const float, d, "rf"); a.ids = GP(int, d, "ids"); a.out = GP(unsigned char, d, "out");
    a.alive = GP(int, d, "alive"); a.probs = GP(float, d, "probs");
    a.N = get<int>(d, "N", 0); a.Bp = get<int>(d, "Bp", 0); a.H = get<int>(d, "H", 0); a.V = get<int>(d, "V", 0);
    a.step = get<int>(d, "step", 0); a.max_len = get<int>(d, "max_len", 0); a.eos = get<int>(d, "eos", 0);
    if (a.Bp % 32 || a.V % 64 || a.V > 512 || a.H % 32) throw std::runtime_error("fc_sample: bad shape");
    fc_sample(a, S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("reduce_slabs", [](uintptr_t src, int splits, long n, uintptr_t dst, uintptr_t s) {
    reduce_slabs(Pp<const float>(src), splits, n, Pp<float>(dst), S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("cast_bf16", [](uintptr_t in, long n, uintptr_t out, uintptr_t s) {
    cast_bf16(Pp<const float>(in), n, Pp<u16>(out), S(s));
    HIP_LAUNCH_CHECK();
  });
  m.def("transpose_bf16", [](uintptr_t in, int R, int C, uintptr_t out, uintptr_t s) {
    transpose_bf16(Pp<const float>(in), R, C, Pp<u16>(out), S(s));
    HIP_LAUNCH_CHECK();
  });

  // ---------------------------------------------------------------- RCCL communicator
  m.def("bootstrap_key", &bootstrap_key);
  m.def("launch_env", [] {
    const LaunchEnv e = launch_env();
    py::dict d;
    d["rank"] = e.rank; d["world"] = e.world; d["local"] = e.local; d["launcher"] = e.launcher;
    return d;
  });
  m.def("bootstrap_path", &bootstrap_path);
  m.def("file_exchange_uid", [](int rank, const std::string& path, const std::string& key, py::bytes uid,
                                int timeout_ms) {
    std::string u = uid;
    py::gil_scoped_release nogil;
    return py::bytes(file_exchange_uid(rank, path, key, u, timeout_ms));
  });
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init([](py::bytes uid, int rank, int world) {
        std::string s = uid;
        return new RcclComm(s, rank, world);
      }))
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      .def("allreduce_avg_f32", [](RcclComm& c, uintptr_t p, long n, uintptr_t s) {
        c.allreduce_avg_f32(Pp<float>(p), n, S(s));
      })
      .def("allreduce_sum_f32", [](RcclComm& c, uintptr_t p, long n, uintptr_t s) {
        c.allreduce_sum_f32(Pp<float>(p), n, S(s));
      })
      .def("allreduce_max_u32", [](RcclComm& c, uintptr_t p, long n, uintptr_t s) {
        c.allreduce_max_u32(Pp<unsigned>(p), n, S(s));
      })
      .def("broadcast_f32", [](RcclComm& c, uintptr_t p, long n, int root, uintptr_t s) {
        c.broadcast_f32(Pp<float>(p), n, root, S(s));
      })
      .def("allgather_u8", [](RcclComm& c, uintptr_t send, uintptr_t recv, long n, uintptr_t s) {
        c.allgather_u8(Pp<const unsigned char>(send), Pp<unsigned char>(recv), n, S(s));
      })
      .def("reduce_scatter_avg_f32", [](RcclComm& c, uintptr_t send, uintptr_t recv, long n, uintptr_t s) {
        c.reduce_scatter_avg_f32(Pp<const float>(send), Pp<float>(recv), n, S(s));
      })
      .def("allgather_f32", [](RcclComm& c, uintptr_t send, uintptr_t recv, long n, uintptr_t s) {
        c.allgather_f32(Pp<const float>(send), Pp<float>(recv), n, S(s));
      })
      .def("count", &RcclComm::count)
      .def("check_async_error", &RcclComm::check_async_error)
      .def("abort", &RcclComm::abort)
      .def("aborted", &RcclComm::aborted)
      .def("rank", &RcclComm::rank)
      .def("world", &RcclComm::world);
}
