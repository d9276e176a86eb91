// jit.hip -- runtime-specialised fused chunk kernels (hipRTC -> gfx950).
//
// The reference composes a pipeline's chunk function at plan time
// (fuse/fuse_multiple, primitive/blockwise.py:368-508) and calls it per
// task.  Here the fused program (cubed_program_t) is compiled once into its
// own gfx950 code object: the generated source instantiates the hand-written
// kernel bodies of kernels.h with
//   * the program bytes as a compile-time constant (every leaf kind, dtype,
//     field rop and output dtype folds), and
//   * the prologue/epilogue as straight-line `sinsn<op, a, b, ...>` calls
//     (vm.h), so registers are named values and no op switch survives.
// The result is the kernel a programmer would write by hand for that chain:
// no interpreter dispatch, no scratch, low register count, high occupancy.
// Code objects are cached per program (by its bytes) for the process and
// loaded once per device on first launch.  Compilation needs no GPU.
#include "fused_common.h"
#include <hip/hiprtc.h>

#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace cubed {

struct JitKernel {
  std::string main_name, fin_name;  // descriptive names (they show in rocprof traces)
  std::string finish_name;          // partials mode: the SoA finish (epilogue after the cross-GPU combine)
  std::string fold_name;            // partials mode: the lifted fold + finish
  std::string source;
  std::string log;
  std::vector<char> code;
  std::mutex mu;
  std::unordered_map<int, hipModule_t> modules;  // per device
  std::unordered_map<int, hipFunction_t> main_fn, fin_fn, finish_fn, fold_fn;
};

static std::mutex g_mu;
static std::unordered_map<std::string, JitKernel*> g_cache;
static int g_stream_force_unroll = 0;  // cubed_stream_force_unroll() (probes: rows in flight per lane)

static void emit_insns(std::string& out, const cubed_insn_t* ins, int n) {
  char buf[160];
  for (int i = 0; i < n; ++i) {
    const cubed_insn_t& I = ins[i];
    snprintf(buf, sizeof(buf), "  sinsn<%d, %d, %d, %d, %d, %d>(regs, P);\n", (int)I.op, (int)I.a,
             (int)I.b, (int)I.c, (int)I.t, (int)I.imm);
    out += buf;
  }
}

static const char* vname(int vtype) {
  return vtype == CUBED_V_F32 ? "float" : vtype == CUBED_V_F64 ? "double" : "int64_t";
}

static const char* vtag(int vtype) {
  return vtype == CUBED_V_F32 ? "f32" : vtype == CUBED_V_F64 ? "f64" : "i64";
}

// e.g. cubed_stream_f32_l2_r1, cubed_map_f64_v4, cubed_reduce_b_f64_v1_r2
std::string jit_kernel_name(const cubed_program_t& P) {
  char buf[96];
  const int kernel = P.mode & 3, vec = (P.mode & 4) ? 4 : 1;
  if (P.mode & CUBED_MODE_STREAM)
    snprintf(buf, sizeof(buf), "cubed_stream_%s_l%d_r%d", vtag(P.vtype), P.nleaves, P.nred);
  else if (P.nfields == 0)
    snprintf(buf, sizeof(buf), "cubed_map_%s_v%d_d%d", vtag(P.vtype), vec, P.ndim);
  else
    snprintf(buf, sizeof(buf), "cubed_reduce_%s_%s_v%d_r%d", kernel == 0 ? "a" : "b", vtag(P.vtype), vec, P.nred);
  std::string s = buf;
  if (P.mode & CUBED_MODE_PARTIALS) s += "_partials";
  // + a digest of the program (FNV-1a over its bytes): every program's
  // kernels carry their own symbol, so a kernel trace separates programs of
  // the same shape (quad-means' mean and the var / std of u*v)
  uint32_t h = 2166136261u;
  const unsigned char* b = (const unsigned char*)&P;
  for (size_t i = 0; i < sizeof(P); ++i) h = (h ^ b[i]) * 16777619u;
  snprintf(buf, sizeof(buf), "_p%08x", h);
  return s + buf;
}

// Partials mode: the SoA finish (cubed_fused_finish_compiled) -- the
// epilogue over combined per-field partials, specialised like the main
// kernel.  The interpreted k_finish_soa walks the program from device memory
// and spent 15-16 us on the 50000 outputs of a rank's rechunk + mean share
// (a short grid of long dependent load chains).
// ... and the lifted fold (cubed_fold_groups_compiled): a full reduction's
// per-element partials folded per group and finished with the program's own
// epilogue -- the interpreted fold's generic combine and epilogue switches
// are the latency chain that kept it at ~40 us for one scalar.
static std::string jit_finish_source(const cubed_program_t& P, const std::string& name) {
  if (!(P.mode & CUBED_MODE_PARTIALS) || P.nfields == 0) return "";
  return "extern \"C\" __global__ __launch_bounds__(256) void " + name +
         "_finish(const cubed_task_t* __restrict__ tasks, int64_t ntasks, int64_t max_kept, "
         "const cubed::Acc* __restrict__ soa, int kd0, int kd1) {\n"
         "  cubed::finish_soa_body(JP, tasks, ntasks, max_kept, soa, kd0, kd1);\n}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void " + name +
         "_fold(const cubed_task_t* __restrict__ tasks, int64_t ntasks, int64_t max_kept, "
         "const cubed::Acc* __restrict__ soa, const int64_t* __restrict__ gs, int64_t ngroups, int64_t nsplit, "
         "cubed::Acc* __restrict__ out_split, cubed::Acc* __restrict__ out, int kd0, int kd1, "
         "const cubed_task_t* __restrict__ fin_tasks) {\n"
         "  if (nsplit > 1)\n"
         "    cubed::fold_groups_split_body<true>(JP, tasks, ntasks, max_kept, soa, gs, ngroups, nsplit, out_split, "
         "out, kd0, kd1, nullptr, fin_tasks);\n"
         "  else\n"
         "    cubed::fold_groups_body<true>(JP, tasks, ntasks, max_kept, soa, gs, ngroups, out, kd0, kd1, nullptr, "
         "fin_tasks);\n}\n";
}

std::string jit_source(const cubed_program_t& P, const std::string& name) {
  std::string s;
  s += "// generated by libcubed_amd (jit.hip) for one fused chunk program\n";
  s += "#define CUBED_RUN_PROLOGUE(V, VEC, regs) jit_prologue<V, VEC>(regs, P)\n";
  s += "#define CUBED_RUN_EPILOGUE(VEC, regs) jit_epilogue<VEC>(regs, P)\n";
  s += "#include \"vm.h\"\nnamespace cubed {\n";
  s += "template <typename V, int VEC>\nCUBED_DEV void jit_prologue(Regs<V, VEC>& regs, const cubed_program_t& P) {\n";
  emit_insns(s, P.insns, P.ninsns);
  s += "}\ntemplate <int VEC>\nCUBED_DEV void jit_epilogue(Regs<double, VEC>& regs, const cubed_program_t& P) {\n";
  emit_insns(s, P.epi, P.nepi > 0 ? P.nepi : 0);
  s += "}\n}  // namespace cubed\n#include \"kernels.h\"\n";
  // the program itself, as constant bytes
  const unsigned char* b = (const unsigned char*)&P;
  s += "namespace cubed_jit {\nalignas(16) static constexpr unsigned char PROG[" +
       std::to_string(sizeof(P)) + "] = {";
  for (size_t i = 0; i < sizeof(P); ++i) {
    s += std::to_string((int)b[i]);
    if (i + 1 < sizeof(P)) s += ",";
  }
  s += "};\n}\n#define JP (reinterpret_cast<const cubed_program_t&>(cubed_jit::PROG))\n";
  const char* V = vname(P.vtype);
  const int kernel = P.mode & 3, vec = (P.mode & 4) ? 4 : 1;
  char buf[512];
  if (P.mode & CUBED_MODE_STREAM) {
    // rows in flight per lane: stream_unroll()'s ~128 B per lane, except f64
    // programs of three or more leaves, where some leaves are usually
    // broadcast over the reduced rows (loaded once, not per row: vorticity's
    // x, y) -- 4 rows there, 1 % faster on vorticity than 2 (3: slower, 8:
    // slower; tools/stream_unroll_probe.py, profiles/r06_stream_unroll.log)
    const int U = g_stream_force_unroll > 0                 ? g_stream_force_unroll
                  : P.vtype == CUBED_V_F64 && P.nleaves >= 3 ? 4
                                                             : stream_unroll(P.vtype == CUBED_V_F32 ? 4 : 8, P.nleaves);
    // the unsplit kernel (a grid that fills the chip without splitting the
    // rows), f32 two-leaf programs: 1 row per lane with W = 4 kept groups
    // (the host's choice for them), 2 rows with W = 2 -- quad-means 1.149-
    // 1.153 ms (W 4, U 1), 1.173-1.179 (W 2, U 2), 1.212-1.215 (W 2, U 4),
    // plans of their own in one process (profiles/r06_stream_unroll.log);
    // the split planner's in-flight estimate (stream_unroll) does not
    // concern unsplit launches
    const int Um = g_stream_force_unroll > 0                      ? U
                   : P.vtype == CUBED_V_F32 && P.nleaves == 2 ? (stream_groups(P) == 4 ? 1 : 2)
                                                                  : U;
    snprintf(buf, sizeof(buf),
             "extern \"C\" __global__ __launch_bounds__(256) void %s(const cubed_task_t* __restrict__ tasks, "
             "int64_t ntasks, int64_t bpt, int32_t nsplit, cubed::Acc* __restrict__ ws, int64_t max_kept) {\n"
             "  cubed::stream_body<%s, %d, %d, %d, false>(JP, tasks, ntasks, bpt, nsplit, ws, max_kept);\n}\n",
             name.c_str(), V, P.nleaves, Um, stream_groups(P));
    s += buf;
    if (P.nfields > 0) {
      // the split variant (nsplit > 1: arrival counters + in-kernel fold)
      snprintf(buf, sizeof(buf),
               "extern \"C\" __global__ __launch_bounds__(256) void %s_split(const cubed_task_t* __restrict__ tasks, "
               "int64_t ntasks, int64_t bpt, int32_t nsplit, cubed::Acc* __restrict__ ws, int64_t max_kept) {\n"
               "  cubed::stream_body<%s, %d, %d, %d, true>(JP, tasks, ntasks, bpt, nsplit, ws, max_kept);\n}\n",
               name.c_str(), V, P.nleaves, U, stream_groups(P));
      s += buf;
    }
    return s + jit_finish_source(P, name);
  } else if (kernel == 0) {
    snprintf(buf, sizeof(buf),
             "extern \"C\" __global__ __launch_bounds__(256) void %s(const cubed_task_t* __restrict__ tasks, "
             "int64_t ntasks, int64_t bpt, int32_t nsplit, cubed::Acc* __restrict__ ws, int64_t max_kept) {\n"
             "  cubed::fused_a_body<%s, %d>(JP, tasks, ntasks, bpt, nsplit, ws, max_kept);\n}\n",
             name.c_str(), V, vec);
  } else {
    snprintf(buf, sizeof(buf),
             "extern \"C\" __global__ __launch_bounds__(256) void %s(const cubed_task_t* __restrict__ tasks, "
             "int64_t ntasks, int64_t max_kept, int32_t nsplit, cubed::Acc* __restrict__ ws) {\n"
             "  cubed::fused_b_body<%s, %d>(JP, tasks, ntasks, max_kept, nsplit, ws);\n}\n",
             name.c_str(), V, vec);
  }
  s += buf;
  if (P.nfields > 0 && !(P.mode & CUBED_MODE_STREAM))
    s += "extern \"C\" __global__ __launch_bounds__(256) void " + name +
         "_finalize(const cubed_task_t* __restrict__ tasks, "
         "int64_t ntasks, int64_t max_kept, int32_t nsplit, const cubed::Acc* __restrict__ ws, int kd0, int kd1) {\n"
         "  cubed::finalize_body(JP, tasks, ntasks, max_kept, nsplit, ws, kd0, kd1);\n}\n";
  return s + jit_finish_source(P, name);
}

static int compile(JitKernel* k, const char* include_dirs) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, k->source.c_str(), "cubed_fused.hip", 0, nullptr, nullptr) !=
      HIPRTC_SUCCESS) {
    set_error("hiprtcCreateProgram failed");
    return CUBED_E_JIT;
  }
  std::vector<std::string> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                                    "-DCUBED_JIT=1"};
  std::string dirs = include_dirs ? include_dirs : "";
  size_t pos = 0;
  while (pos <= dirs.size()) {
    size_t e = dirs.find(';', pos);
    if (e == std::string::npos) e = dirs.size();
    if (e > pos) opts.push_back("-I" + dirs.substr(pos, e - pos));
    pos = e + 1;
  }
  std::vector<const char*> argv;
  for (auto& o : opts) argv.push_back(o.c_str());
  hiprtcResult r = hiprtcCompileProgram(prog, (int)argv.size(), argv.data());
  size_t n = 0;
  hiprtcGetProgramLogSize(prog, &n);
  k->log.assign(n, '\0');
  if (n) hiprtcGetProgramLog(prog, &k->log[0]);
  if (r != HIPRTC_SUCCESS) {
    std::string msg = "hipRTC compile of a fused program failed: " + k->log.substr(0, 400);
    set_error(msg.c_str());
    hiprtcDestroyProgram(&prog);
    return CUBED_E_JIT;
  }
  hiprtcGetCodeSize(prog, &n);
  k->code.resize(n);
  hiprtcGetCode(prog, k->code.data());
  hiprtcDestroyProgram(&prog);
  return 0;
}

static int load(JitKernel* k, hipStream_t stream, hipFunction_t* main_fn, hipFunction_t* fin_fn) {
  int dev = 0;
  hipError_t e = stream ? hipStreamGetDevice(stream, &dev) : hipGetDevice(&dev);
  if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
  std::lock_guard<std::mutex> g(k->mu);
  auto it = k->modules.find(dev);
  if (it == k->modules.end()) {
    hipModule_t m;
    e = hipModuleLoadData(&m, k->code.data());
    if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
    hipFunction_t f0 = nullptr, f1 = nullptr;
    e = hipModuleGetFunction(&f0, m, k->main_name.c_str());
    if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
    if (hipModuleGetFunction(&f1, m, k->fin_name.c_str()) != hipSuccess) f1 = nullptr;
    hipFunction_t f2 = nullptr, f3 = nullptr;
    if (hipModuleGetFunction(&f2, m, k->finish_name.c_str()) != hipSuccess) f2 = nullptr;
    if (hipModuleGetFunction(&f3, m, k->fold_name.c_str()) != hipSuccess) f3 = nullptr;
    (void)hipGetLastError();
    k->modules[dev] = m;
    k->main_fn[dev] = f0;
    k->fin_fn[dev] = f1;
    k->finish_fn[dev] = f2;
    k->fold_fn[dev] = f3;
  }
  *main_fn = k->main_fn[dev];
  *fin_fn = k->fin_fn[dev];
  return 0;
}

}  // namespace cubed

using namespace cubed;

extern "C" int cubed_fused_compile(const cubed_program_t* prog, const char* include_dirs,
                                   void** handle) {
  if (!prog || !handle) { set_error("cubed_fused_compile: null argument"); return CUBED_E_ARG; }
  if (int rc = check_program(*prog)) return rc;
  std::string key((const char*)prog, sizeof(*prog));
  key += std::to_string(g_stream_force_unroll);
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_cache.find(key);
    if (it != g_cache.end()) { *handle = it->second; return 0; }
  }
  JitKernel* k = new JitKernel();
  k->main_name = jit_kernel_name(*prog);
  k->fin_name = k->main_name + ((prog->mode & CUBED_MODE_STREAM) ? "_split" : "_finalize");
  k->finish_name = k->main_name + "_finish";
  k->fold_name = k->main_name + "_fold";
  k->source = jit_source(*prog, k->main_name);
  if (int rc = compile(k, include_dirs)) { delete k; return rc; }
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_cache.find(key);
  if (it != g_cache.end()) { delete k; *handle = it->second; return 0; }
  g_cache[key] = k;
  *handle = k;
  return 0;
}

extern "C" const char* cubed_fused_source(const void* handle) {
  return handle ? ((const JitKernel*)handle)->source.c_str() : "";
}

extern "C" int64_t cubed_fused_code_bytes(const void* handle) {
  return handle ? (int64_t)((const JitKernel*)handle)->code.size() : 0;
}

extern "C" int cubed_fused_chunks_compiled(void* handle, const cubed_program_t* prog,
                                           const cubed_program_t* d_prog, const cubed_task_t* d_tasks,
                                           int64_t ntasks, int64_t max_kept, int64_t max_red,
                                           void* d_workspace, int64_t workspace_bytes, void* stream) {
  if (!handle || !prog || (!d_tasks && ntasks > 0)) {
    set_error("cubed_fused_chunks_compiled: null argument");
    return CUBED_E_ARG;
  }
  if (ntasks == 0) return 0;
  const cubed_program_t& P = *prog;
  if (int rc = check_program(P)) return rc;
  if (max_kept <= 0 || max_red <= 0) { set_error("cubed_fused_chunks_compiled: empty task bounds"); return CUBED_E_ARG; }
  const LaunchPlan L = plan_launch(&P, ntasks, max_kept, max_red,
                                   (P.mode & CUBED_MODE_STREAM) ? stream_groups(P) : 1);
  if (L.ws_bytes > 0 && (d_workspace == nullptr || workspace_bytes < L.ws_bytes)) {
    set_error("cubed_fused_chunks_compiled: workspace too small");
    return CUBED_E_WORKSPACE;
  }
  if (!owner_major_fits(P, L.soa_elems)) {
    set_error("cubed_fused_chunks_compiled: owner-major slots exceed the SoA block");
    return CUBED_E_ARG;
  }
  hipFunction_t fmain = nullptr, ffin = nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (int rc = load((JitKernel*)handle, st, &fmain, &ffin)) return rc;
  Acc* ws = (Acc*)d_workspace + L.soa_elems;  // partials mode: SoA block first
  const dim3 grid = grid_of(L.blocks);
  hipError_t e;
  int32_t nsplit = L.nsplit;
  int64_t bpt = L.bpt;
  const cubed_task_t* tasks = d_tasks;
  if ((P.mode & CUBED_MODE_STREAM) && L.nsplit > 1) {
    // split streaming reduction: the _split variant folds in-kernel
    if (!ffin) { set_error("cubed_fused_chunks_compiled: no split kernel"); return CUBED_E_JIT; }
    if (L.balanced) nsplit = -nsplit;  // stream_body's balanced split
    void* args[] = {&tasks, &ntasks, &bpt, &nsplit, &ws, &max_kept};
    e = hipModuleLaunchKernel(ffin, grid.x, grid.y, 1, kBlock, 1, 1, 0, st, args, nullptr);
    if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
    return 0;
  }
  if (L.kernel == 0) {
    void* args[] = {&tasks, &ntasks, &bpt, &nsplit, &ws, &max_kept};
    e = hipModuleLaunchKernel(fmain, grid.x, grid.y, 1, kBlock, 1, 1, 0, st, args, nullptr);
  } else {
    void* args[] = {&tasks, &ntasks, &max_kept, &nsplit, &ws};
    e = hipModuleLaunchKernel(fmain, grid.x, grid.y, 1, kBlock, 1, 1, 0, st, args, nullptr);
  }
  if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
  // streaming kernels fold their splits and write SoA partials themselves
  if (P.mode & CUBED_MODE_STREAM) return 0;
  if (P.mode & CUBED_MODE_PARTIALS) {
    if (!d_prog) { set_error("cubed_fused_chunks_compiled: partials mode needs d_prog"); return CUBED_E_ARG; }
    return launch_collect(P, d_prog, L, d_tasks, ntasks, max_kept, (Acc*)d_workspace, st);
  }
  if (L.nsplit > 1) {
    if (!ffin) { set_error("cubed_fused_chunks_compiled: no finalize kernel"); return CUBED_E_JIT; }
    int kd0 = (L.kernel == 0) ? P.nred : 0;
    int kd1 = (L.kernel == 0) ? P.ndim : P.ndim - P.nred;
    const int64_t n = ntasks * max_kept;
    const dim3 g2 = grid_of((n + kBlock - 1) / kBlock);
    const Acc* cws = ws;
    void* args[] = {&tasks, &ntasks, &max_kept, &nsplit, &cws, &kd0, &kd1};
    e = hipModuleLaunchKernel(ffin, g2.x, g2.y, 1, kBlock, 1, 1, 0, st, args, nullptr);
    if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
  }
  return 0;
}

extern "C" int cubed_fused_finish_compiled(void* handle, const cubed_program_t* prog, const cubed_task_t* d_tasks,
                                           int64_t ntasks, int64_t max_kept, const void* d_partials,
                                           void* stream) {
  if (!handle || !prog || !d_partials || (!d_tasks && ntasks > 0)) {
    set_error("cubed_fused_finish_compiled: null argument");
    return CUBED_E_ARG;
  }
  if (ntasks == 0) return 0;
  if (int rc = check_program(*prog)) return rc;
  if (!(prog->mode & CUBED_MODE_PARTIALS) || prog->nfields == 0 || max_kept <= 0) {
    set_error("cubed_fused_finish_compiled: not a partials-mode reduction");
    return CUBED_E_ARG;
  }
  JitKernel* k = (JitKernel*)handle;
  hipFunction_t fmain = nullptr, ffin = nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (int rc = load(k, st, &fmain, &ffin)) return rc;
  hipFunction_t ff;
  {
    int dev = 0;
    hipError_t e = st ? hipStreamGetDevice(st, &dev) : hipGetDevice(&dev);
    if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
    std::lock_guard<std::mutex> g(k->mu);
    ff = k->finish_fn[dev];
  }
  if (!ff) { set_error("cubed_fused_finish_compiled: the program has no finish kernel"); return CUBED_E_JIT; }
  int kd0, kd1;
  kept_dims(*prog, kd0, kd1);
  const int64_t n = ntasks * max_kept;
  const dim3 grid = grid_of((n + kBlock - 1) / kBlock);
  const Acc* soa = (const Acc*)d_partials;
  const cubed_task_t* tasks = d_tasks;
  void* args[] = {&tasks, &ntasks, &max_kept, &soa, &kd0, &kd1};
  hipError_t e = hipModuleLaunchKernel(ff, grid.x, grid.y, 1, kBlock, 1, 1, 0, st, args, nullptr);
  if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
  return 0;
}

extern "C" int cubed_fold_groups_compiled(void* handle, const cubed_program_t* prog, const cubed_task_t* d_tasks,
                                          int64_t ntasks, int64_t max_kept, const void* d_row_partials,
                                          const int64_t* d_group_start, int64_t ngroups, void* d_group_partials,
                                          int64_t nsplit, void* d_split_ws, const cubed_task_t* d_fin_tasks,
                                          void* stream) {
  if (!handle || !prog || !d_row_partials || !d_group_start || !d_group_partials || !d_fin_tasks ||
      (!d_tasks && ntasks > 0) || (nsplit > 1 && !d_split_ws)) {
    set_error("cubed_fold_groups_compiled: null argument");
    return CUBED_E_ARG;
  }
  if (ngroups == 0) return 0;
  if (int rc = check_program(*prog)) return rc;
  if (!(prog->mode & CUBED_MODE_PARTIALS) || prog->nfields == 0 || max_kept <= 0 || ngroups > ntasks ||
      nsplit < 1) {
    set_error("cubed_fold_groups_compiled: not a partials-mode reduction / bad shape");
    return CUBED_E_ARG;
  }
  JitKernel* k = (JitKernel*)handle;
  hipFunction_t fmain = nullptr, ffin = nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (int rc = load(k, st, &fmain, &ffin)) return rc;
  hipFunction_t ff;
  {
    int dev = 0;
    hipError_t e = st ? hipStreamGetDevice(st, &dev) : hipGetDevice(&dev);
    if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
    std::lock_guard<std::mutex> g(k->mu);
    ff = k->fold_fn[dev];
  }
  if (!ff) { set_error("cubed_fold_groups_compiled: the program has no fold kernel"); return CUBED_E_JIT; }
  int kd0, kd1;
  kept_dims(*prog, kd0, kd1);
  const dim3 grid = grid_of(ngroups * nsplit);
  const cubed_task_t* tasks = d_tasks;
  const Acc* soa = (const Acc*)d_row_partials;
  const int64_t* gs = d_group_start;
  Acc* out_split = (Acc*)d_split_ws;
  Acc* out = (Acc*)d_group_partials;
  const cubed_task_t* fin_tasks = d_fin_tasks;
  void* args[] = {&tasks, &ntasks, &max_kept, &soa, &gs, &ngroups, &nsplit, &out_split, &out, &kd0, &kd1, &fin_tasks};
  hipError_t e = hipModuleLaunchKernel(ff, grid.x, grid.y, 1, kBlock, 1, 1, 0, st, args, nullptr);
  if (e != hipSuccess) { set_error(hipGetErrorString(e)); return (int)e; }
  return 0;
}

// Probes only (tools/stream_unroll_probe.py): rows in flight per lane of the
// JIT streaming kernels compiled from now on (0 = stream_unroll()'s choice);
// returns the previous value.  Not part of the C ABI header.
extern "C" int cubed_stream_force_unroll(int u) {
  std::lock_guard<std::mutex> g(g_mu);
  const int prev = g_stream_force_unroll;
  if (u >= 0) g_stream_force_unroll = u;
  return prev;
}
