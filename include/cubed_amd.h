/*
 * cubed_amd.h -- C ABI of the MI355X execution path for Cubed's blockwise /
 * reduction / rechunk primitives (libcubed_amd.so).
 *
 * Plain C: fixed-size structs, raw device pointers, element counts and a
 * hipStream_t passed as void*.  No torch or C++ types cross this boundary.
 * The caller owns every buffer (arrays, task tables, workspace); the library
 * never allocates or frees persistent memory and never synchronises the
 * device.  Every entry point returns 0 on success, a positive hipError_t
 * value on a HIP failure, or a negative CUBED_E_* code on a bad argument;
 * cubed_last_error() gives a message for the calling thread.
 *
 * Which reference interface each entry point replaces (paths relative to the
 * reference tree, rsignell/cubed v0.12.0):
 *
 *   cubed_fused_chunks   -> apply_blockwise(out_key, config=BlockwiseSpec)
 *                           cubed/primitive/blockwise.py:61-84, running the
 *                           fused chunk function built by fuse/fuse_multiple
 *                           (:368-508): elementwise chains (array_object.py
 *                           :121-348, elementwise_functions.py), per-chunk
 *                           reductions (_mean_func/_mean_combine/
 *                           _mean_aggregate statistical_functions.py:54-100,
 *                           nan_functions.py:37-59, sum/max/min/prod) and the
 *                           merge_chunks+combine rounds of core/ops.py:849-889.
 *   cubed_random_chunks  -> _random(x, numblocks, root_seed, block_id)
 *                           cubed/random.py:31-36 (numpy Philox4x64-10 +
 *                           Generator.random), bit-exact.
 *   cubed_copy_boxes     -> copy_read_to_write(chunk_key, config=CubedCopySpec)
 *                           cubed/primitive/rechunk.py:187-192, and the
 *                           map_direct region reads _copy_chunk
 *                           (core/ops.py:784-787) / _read_index_chunk
 *                           (core/ops.py:481-486).
 *   cubed_gemm_chain     -> _matmul / _tensordot chunk products together
 *                           with the _sum_wo_cat k-sum
 *                           cubed/array_api/linear_algebra_functions.py
 *                           :35-78, :139-149 (numpy BLAS sgemm/dgemm per task
 *                           + a reduction over k).
 */
#ifndef CUBED_AMD_H
#define CUBED_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CUBED_ABI_VERSION 16

#define CUBED_MAX_DIMS 6   /* iteration dims of one task after coalescing   */
#define CUBED_MAX_LEAVES 4 /* array/philox/const-array inputs of a program  */
#define CUBED_MAX_FIELDS 3 /* reduced fields (mean: n, total; var: n, mu, M2) */
#define CUBED_MAX_OUTS 3   /* output arrays written per task (var: n, mu, M2) */
#define CUBED_MAX_INSNS 48 /* VM instructions in the prologue program       */
#define CUBED_MAX_EPI 16   /* VM instructions in the epilogue program       */
#define CUBED_MAX_CONSTS 16
#define CUBED_NREGS 6      /* VM registers; leaf i is preloaded into reg i  */

/* error codes (negative); positive values are hipError_t */
#define CUBED_MODE_STREAM 8
#define CUBED_MODE_PARTIALS 16
#define CUBED_MODE_STREAM_W2 32
#define CUBED_MODE_STREAM_W4 64
#define CUBED_MODE_HOST_COUNT 128 /* partials: COUNT fields are left to the host */
#define CUBED_MODE_STREAM_EVEN 256 /* stream: every task the same reduced extent */
/* stream + partials, multi-GPU reduce-scatter (ABI 16): the ONE stored field's
 * partial of SoA element i (group g = i / mko) is written to owner-major slot
 * ((g % W) * L + g / W) * mko + i % mko of the SoA region, with mko, W, L in
 * consts[CUBED_MAX_CONSTS - 3 .. - 1] (host-checked: block-cyclic owners, one
 * summed field, every other field host-counted) */
#define CUBED_MODE_OWNER_MAJOR 512

#define CUBED_E_ARG (-1)
#define CUBED_E_DTYPE (-2)
#define CUBED_E_LAYOUT (-3)
#define CUBED_E_WORKSPACE (-4)
#define CUBED_E_JIT (-5)
#define CUBED_E_CODEC (-6)       /* malformed compressed chunk */
#define CUBED_E_UNSUPPORTED (-7) /* codec / shuffle this build does not decode */

/* element dtypes (numpy kinds); bool is 1 byte 0/1 */
enum cubed_dtype {
  CUBED_BOOL = 0, CUBED_I8, CUBED_I16, CUBED_I32, CUBED_I64,
  CUBED_U8, CUBED_U16, CUBED_U32, CUBED_U64,
  CUBED_F32, CUBED_F64, CUBED_F16, CUBED_BF16
};

/* register value type of a program (all arithmetic happens in it; narrower
 * node dtypes are re-rounded by CAST instructions) */
enum cubed_vtype { CUBED_V_F32 = 0, CUBED_V_F64 = 1, CUBED_V_I64 = 2 };

/* leaf kinds */
enum cubed_leaf_kind {
  CUBED_LEAF_ARRAY = 0,  /* strided view of a chunk (or of merged chunks)  */
  CUBED_LEAF_PHILOX = 1, /* numpy Generator(Philox(key)).random() stream,  */
                         /* element = C-order position in the task's box   */
  CUBED_LEAF_OFFSET = 2, /* the task's block offset (int64), for block_id  */
  CUBED_LEAF_IOTA = 3    /* int64 value leaf_base + sum(coord*stride): the  */
                         /* global index along an axis (arange/eye/tril)    */
};

/* reduction ops of a field; accumulators are f64 or i64 (acc_type).  The
 * pair ops couple field 0 (the lead, one of ARGMAX/ARGMIN/CPROD) with field 1
 * (its partner, PAIR_INDEX / PAIR_IMAG): argmax/argmin reduce {value, index}
 * pairs (core/ops.py:1093-1153 _arg_func/_arg_combine), cprod the {re, im}
 * parts of a complex product (np.prod of complex chunks).  A program holding
 * a pair has exactly these two fields.
 * var triples couple field 0 (n, int64: VAR or VARC) with field 1 (mu,
 * VAR_MEAN) and field 2 (M2, VAR_M2), f64: the count, mean and sum of
 * squared deviations of Chan, Golub & LeVeque's pairwise update.  VAR folds
 * element VALUES (field 0's source) by Welford's update; VARC folds partial
 * {n, mu, M2} triples (the three fields' sources) -- the combine rounds of
 * var's reduction; accumulators always combine by Chan's update.  A program
 * holding a triple has exactly these three fields. */
enum cubed_rop {
  CUBED_R_NONE = 0, CUBED_R_SUM, CUBED_R_NANSUM, CUBED_R_COUNT,
  CUBED_R_COUNT_NONNAN, CUBED_R_MAX, CUBED_R_MIN, CUBED_R_PROD,
  CUBED_R_NANMAX, CUBED_R_NANMIN, CUBED_R_ANY, CUBED_R_ALL, CUBED_R_NANPROD,
  CUBED_R_ARGMAX, CUBED_R_ARGMIN, CUBED_R_CPROD, CUBED_R_PAIR_INDEX, CUBED_R_PAIR_IMAG,
  CUBED_R_VAR, CUBED_R_VARC, CUBED_R_VAR_MEAN, CUBED_R_VAR_M2
};

/* VM opcodes (two-address: r[a] = op(r[a], r[b]); where: r[a] = r[c] ? r[a] : r[b]) */
enum cubed_op {
  CUBED_OP_NOP = 0,
  CUBED_OP_CONST,   /* r[a] = consts[imm]                                  */
  CUBED_OP_MOV,     /* r[a] = r[b]                                         */
  CUBED_OP_CAST,    /* r[a] = round r[a] to dtype t (from dtype imm)       */
  CUBED_OP_WHERE,   /* r[a] = r[c] ? r[a] : r[b]                           */
  /* unary */
  CUBED_OP_NEG = 16, CUBED_OP_ABS, CUBED_OP_SQRT, CUBED_OP_EXP, CUBED_OP_LOG,
  CUBED_OP_SIN, CUBED_OP_COS, CUBED_OP_TAN, CUBED_OP_TANH, CUBED_OP_FLOOR,
  CUBED_OP_CEIL, CUBED_OP_TRUNC, CUBED_OP_RINT, CUBED_OP_ISNAN, CUBED_OP_ISINF,
  CUBED_OP_ISFINITE, CUBED_OP_LNOT, CUBED_OP_BNOT, CUBED_OP_SIGN,
  CUBED_OP_SQUARE, CUBED_OP_RECIP, CUBED_OP_LOG1P, CUBED_OP_EXPM1,
  CUBED_OP_LOG2, CUBED_OP_LOG10, CUBED_OP_SINH, CUBED_OP_COSH, CUBED_OP_ASIN,
  CUBED_OP_ACOS, CUBED_OP_ATAN, CUBED_OP_ASINH, CUBED_OP_ACOSH,
  CUBED_OP_ATANH, CUBED_OP_EXP2, CUBED_OP_SIGNBIT,
  /* binary */
  CUBED_OP_ADD = 64, CUBED_OP_SUB, CUBED_OP_MUL, CUBED_OP_DIV,
  CUBED_OP_FLOORDIV, CUBED_OP_MOD, CUBED_OP_POW, CUBED_OP_MAX, CUBED_OP_MIN,
  CUBED_OP_EQ, CUBED_OP_NE, CUBED_OP_LT, CUBED_OP_LE, CUBED_OP_GT,
  CUBED_OP_GE, CUBED_OP_LAND, CUBED_OP_LOR, CUBED_OP_LXOR, CUBED_OP_BAND,
  CUBED_OP_BOR, CUBED_OP_BXOR, CUBED_OP_SHL, CUBED_OP_SHR, CUBED_OP_ATAN2,
  CUBED_OP_HYPOT, CUBED_OP_LOGADDEXP, CUBED_OP_COPYSIGN, CUBED_OP_FMAX,
  CUBED_OP_FMIN, CUBED_OP_LOGADDEXP2
};

typedef struct {
  uint8_t op, a, b, c; /* opcode and register operands                      */
  uint8_t t;           /* CAST target dtype                                 */
  uint8_t pad;
  uint16_t imm;        /* CONST index / CAST source dtype                   */
} cubed_insn_t;

/* A fused chunk program: leaves -> prologue -> (per-field reduce) ->
 * epilogue -> outputs.  Passed by value as the kernel argument. */
typedef struct {
  int32_t vtype;                 /* enum cubed_vtype                        */
  int32_t ndim;                  /* iteration dims (<= CUBED_MAX_DIMS)      */
  int32_t nred;                  /* dims [0,nred) are reduced (kernel A) or */
                                 /* dims [ndim-nred,ndim) (kernel B)        */
  int32_t mode;                  /* kernel shape: 0 = A (reduced dims first,*/
                                 /* or a map), 1 = B (reduced dims last);   */
                                 /* +4 when the innermost dim is packed     */
                                 /* (VEC=4 loads/stores; host-checked)      */
                                 /* +8 (CUBED_MODE_STREAM): streaming fast  */
                                 /* path, host-checked: kernel A, VEC=4,    */
                                 /* ndim == nred + 1, nred <= 2, every leaf */
                                 /* an ARRAY in the vtype's own dtype       */
                                 /* (f32/f64/i64) with packed kept dim and  */
                                 /* reduced strides that are multiples of 4 */
                                 /* +16 (CUBED_MODE_PARTIALS): reductions   */
                                 /* stop before the epilogue and leave the  */
                                 /* per-field accumulators as SoA partials  */
                                 /* at the start of the workspace (see      */
                                 /* cubed_fused_finish)                     */
                                 /* +32 / +64 (CUBED_MODE_STREAM_W2 / _W4): */
                                 /* streaming JIT kernels give each thread  */
                                 /* 2 / 4 groups of 4 kept elements         */
                                 /* (interpreted kernels ignore the bits)   */
                                 /* +128 (CUBED_MODE_HOST_COUNT): partials  */
                                 /* mode leaves plain COUNT fields unwritten*/
                                 /* in the SoA block -- the host fills them */
                                 /* with the (geometry-known) global count  */
                                 /* +256 (CUBED_MODE_STREAM_EVEN), +512     */
                                 /* (CUBED_MODE_OWNER_MAJOR): see above     */
  int32_t nleaves;
  uint8_t leaf_kind[CUBED_MAX_LEAVES];
  uint8_t leaf_dtype[CUBED_MAX_LEAVES];
  int32_t nfields;               /* 0 = map (no reduction)                  */
  uint8_t field_rop[CUBED_MAX_FIELDS];
  uint8_t field_acc[CUBED_MAX_FIELDS]; /* 0 = f64 accumulator, 1 = i64     */
  uint8_t field_src[CUBED_MAX_FIELDS]; /* register holding the field value  */
  uint8_t pad0[3];
  int32_t nouts;
  uint8_t out_dtype[CUBED_MAX_OUTS];
  uint8_t out_src[CUBED_MAX_OUTS]; /* register (or field when no epilogue)  */
  uint8_t pad1[2];
  int32_t ninsns;
  int32_t nepi;                  /* -1 = store fields directly              */
  cubed_insn_t insns[CUBED_MAX_INSNS];
  cubed_insn_t epi[CUBED_MAX_EPI];
  union { double f; int64_t i; } consts[CUBED_MAX_CONSTS];
} cubed_program_t;

/* One task (= one output chunk of the pipeline, or one sub-box of it).
 * Strides are in elements; a broadcast dim has stride 0; an output has
 * stride 0 on reduced dims.  Bases are device byte addresses. */
typedef struct {
  int64_t extent[CUBED_MAX_DIMS];
  int64_t leaf_base[CUBED_MAX_LEAVES];
  int64_t leaf_stride[CUBED_MAX_LEAVES][CUBED_MAX_DIMS];
  int64_t out_base[CUBED_MAX_OUTS];
  int64_t out_stride[CUBED_MAX_OUTS][CUBED_MAX_DIMS];
  uint64_t key_lo, key_hi; /* Philox key of this task's random leaf          */
  int64_t block_offset;    /* C-order block offset (block_id_to_offset)      */
  int64_t pad;
} cubed_task_t;

/* Run a fused chunk program over ntasks tasks (task table in device memory).
 * All tasks share the dim structure of `prog` (ndim, nred) but may differ in
 * extents (edge chunks).  max_kept / max_red bound the per-task kept and
 * reduced element counts (the library sizes its grid from them).
 * `prog` is read on the host (launch shape, argument checks); `d_prog` is a
 * byte-identical copy in device memory that the kernels read through the
 * scalar cache (a by-value kernel argument indexed by the interpreter loop
 * would be demoted to scratch).
 * workspace may be NULL when cubed_fused_workspace_bytes() returns 0. */
int cubed_fused_chunks(const cubed_program_t* prog, const cubed_program_t* d_prog,
                       const cubed_task_t* d_tasks,
                       int64_t ntasks, int64_t max_kept, int64_t max_red,
                       void* d_workspace, int64_t workspace_bytes, void* stream);

/* Runtime-specialised form of cubed_fused_chunks (same semantics, same task
 * table): cubed_fused_compile() generates a kernel for *prog with the program
 * baked in as compile-time constants (straight-line code, no interpreter
 * dispatch), compiles it for gfx950 with hipRTC and caches the code object
 * per program for the life of the process.  `include_dirs` is a ';'-separated
 * list holding kernels.h/vm.h/common.h and cubed_amd.h.  Needs no GPU; the
 * code object is loaded on the current device at first launch.
 * Replaces the same reference interface as cubed_fused_chunks, plus the
 * plan-time composition of the chunk function (fuse / fuse_multiple,
 * cubed/primitive/blockwise.py:368-508). */
int cubed_fused_compile(const cubed_program_t* prog, const char* include_dirs, void** handle);
int cubed_fused_chunks_compiled(void* handle, const cubed_program_t* prog,
                                const cubed_program_t* d_prog, const cubed_task_t* d_tasks,
                                int64_t ntasks, int64_t max_kept, int64_t max_red,
                                void* d_workspace, int64_t workspace_bytes, void* stream);
/* The generated source / code object size of a compiled program (diagnostics). */
const char* cubed_fused_source(const void* handle);
int64_t cubed_fused_code_bytes(const void* handle);

/* Split target of streaming reductions: a grid too small to cover HBM
 * latency unsplit is split toward this many workgroups (default 256, one per
 * CU).  Process-wide tuning hook for probes (tools/); workgroups <= 0 only
 * queries.  Returns the previous value. */
int64_t cubed_stream_split_target(int64_t workgroups);
/* Probe hook: split streaming reductions whose grid already fills the chip
 * into nsplit row ranges too (0 = off, the default; < 0 queries). */
int64_t cubed_stream_force_split(int64_t nsplit);

/* Workspace the call above needs (split reductions keep partial
 * accumulators there).  Pure host function. */
int64_t cubed_fused_workspace_bytes(const cubed_program_t* prog, int64_t ntasks,
                                    int64_t max_kept, int64_t max_red);

/* Multi-GPU reductions (partials mode, CUBED_MODE_PARTIALS in prog->mode).
 * cubed_fused_chunks / _compiled then stop before the epilogue: the first
 * nfields*ntasks*max_kept*8 bytes of the workspace receive the per-field
 * accumulators as SoA, partials[f][t][k] (f64 or i64 per field_acc, the
 * reduction identity for k past an edge task's extent), identical in layout
 * on every rank so they can be combined with RCCL.  Replaces the last
 * combine round + aggregate of reduction (cubed/core/ops.py:849-892,
 * _mean_combine/_mean_aggregate statistical_functions.py:61-100) when the
 * round's inputs live on different GPUs.
 * cubed_fused_finish runs the epilogue + stores of the same program from
 * combined SoA partials (same task table, ntasks, max_kept).
 * cubed_combine_partials folds nparts SoA blocks (nfields*n accumulators
 * each, n = ntasks*max_kept, block r at r*nfields*n) in block order into
 * d_out with the fields' own combine ops (used for max/min/prod/any/all,
 * whose NaN semantics RCCL's reductions do not follow). */
int cubed_fused_finish(const cubed_program_t* prog, const cubed_program_t* d_prog,
                       const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept,
                       const void* d_partials, void* stream);
/* The same finish, specialised: the JIT module of `handle` (cubed_fused_compile
 * of a CUBED_MODE_PARTIALS program) carries it; CUBED_E_JIT if it does not. */
int cubed_fused_finish_compiled(void* handle, const cubed_program_t* prog, const cubed_task_t* d_tasks,
                                int64_t ntasks, int64_t max_kept, const void* d_partials, void* stream);
/* Grouped finish (partials mode): tasks [group_start[g], group_start[g+1]) are
 * pieces of ONE output box -- a task split where its inputs straddle source
 * chunks along a reduced dim (e.g. the a[1:] regions of index/map_direct,
 * core/ops.py:374-486, feeding a reduction) -- whose partials are combined in
 * piece order; the first piece's output views get the epilogue.
 * d_group_start: ngroups + 1 int64 in device memory. */
int cubed_fused_finish_groups(const cubed_program_t* prog, const cubed_program_t* d_prog,
                              const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept,
                              const void* d_partials, const int64_t* d_group_start,
                              int64_t ngroups, void* stream);
/* Multi-GPU form of the grouped finish: fold each group's rows into
 * d_group_partials[f][g][k] (max_kept_out per group, identity past a group's
 * kept extent) WITHOUT the epilogue, so the per-rank group partials -- pieces
 * of one output box run on the GPUs that hold their source chunks -- can be
 * combined over RCCL and finished by cubed_fused_finish on the owner. */
int cubed_combine_groups(const cubed_program_t* prog, const cubed_program_t* d_prog,
                         const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept,
                         const void* d_row_partials, const int64_t* d_group_start,
                         int64_t ngroups, int64_t max_kept_out, void* d_group_partials,
                         void* stream);
/* Fold each group's rows AND their kept elements into one accumulator per
 * field: d_group_partials[f][g].  For full reductions run "lifted" (the
 * innermost reduced dims walked as kept dims so every lane streams, e.g.
 * mean(a[1:] * x + b[1:] * y) of the vorticity example).  With an epilogue
 * program (fin / d_fin: the same program with nred = ndim) the kernel also
 * finishes each group into d_fin_tasks[g] (one launch); without it the caller
 * runs cubed_fused_finish over d_group_partials.  ABI 13. */
int cubed_fold_groups(const cubed_program_t* prog, const cubed_program_t* d_prog,
                      const cubed_task_t* d_tasks, int64_t ntasks, int64_t max_kept,
                      const void* d_row_partials, const int64_t* d_group_start,
                      int64_t ngroups, void* d_group_partials, int64_t nsplit,
                      void* d_split_ws, const cubed_program_t* fin, const cubed_program_t* d_fin,
                      const cubed_task_t* d_fin_tasks, void* stream);
/* Splits per group cubed_fold_groups should use (few groups of many
 * elements: each group's rows x max_kept SoA entries cut into nsplit equal
 * runs, the last run to finish folds them); d_split_ws then holds
 * nfields x ngroups x nsplit 8-byte accumulators followed by ngroups uint32
 * arrival counters -- zero it once, the kernel leaves the counters at zero. */
int64_t cubed_fold_groups_splits(int64_t ngroups, int64_t max_rows_per_group, int64_t max_kept);
/* The same fold + finish from the JIT module of a CUBED_MODE_PARTIALS program
 * (cubed_fused_compile): combine and epilogue specialised, the epilogue the
 * program's own (its outputs through d_fin_tasks[g]); CUBED_E_JIT if the
 * module has no fold kernel. */
int cubed_fold_groups_compiled(void* handle, const cubed_program_t* prog, const cubed_task_t* d_tasks,
                               int64_t ntasks, int64_t max_kept, const void* d_row_partials,
                               const int64_t* d_group_start, int64_t ngroups, void* d_group_partials,
                               int64_t nsplit, void* d_split_ws, const cubed_task_t* d_fin_tasks, void* stream);
int cubed_combine_partials(const cubed_program_t* prog, const cubed_program_t* d_prog,
                           const void* d_parts, int32_t nparts, int64_t n, void* d_out,
                           void* stream);
/* Fill ntasks chunks with numpy Generator(Philox(key)).random() doubles:
 * d_out[i] (device pointers) gets counts[i] doubles from key (lo,hi)[i].
 * All three tables are device arrays of ntasks entries. */
int cubed_random_chunks(const int64_t* d_out_ptrs, const int64_t* d_counts,
                        const uint64_t* d_keys /* 2*ntasks: lo,hi */,
                        int64_t ntasks, int64_t max_count, void* stream);

/* Strided N-d box copies (rechunk, merge_chunks, index).  Each box moves
 * extent[0..ndim) elements of `itemsize` bytes from src to dst views. */
typedef struct {
  int64_t src_base, dst_base;      /* device byte addresses                 */
  int64_t extent[CUBED_MAX_DIMS];  /* innermost last; unused dims = 1       */
  int64_t src_stride[CUBED_MAX_DIMS];
  int64_t dst_stride[CUBED_MAX_DIMS];
} cubed_box_t;

/* path: CUBED_COPY_ROWS   -- innermost dim contiguous on both sides; rows are
 *                            moved with lane_bytes-wide lanes (16/8/4/1, must
 *                            divide every row's byte count and offset);
 *                            work = max rows per box, row_bytes = max row size
 *       CUBED_COPY_ELEMS  -- any strides, element at a time; work = max elems
 *       CUBED_COPY_TILE   -- 2-d boxes, src contiguous along dim 1 and dst
 *                            along dim 0 (64x64 LDS tile); work = tiles/box
 *       CUBED_COPY_FLAT   -- 2-d boxes, innermost dim contiguous on both sides
 *                            and dst packed (dst_stride[0] == extent[1]): the
 *                            box is written as one run of lane_bytes words;
 *                            work = max words per box (< 2^31) */
#define CUBED_COPY_ROWS 0
#define CUBED_COPY_ELEMS 1
#define CUBED_COPY_TILE 2
#define CUBED_COPY_FLAT 3
int cubed_copy_boxes(const cubed_box_t* d_boxes, int64_t nboxes, int32_t ndim,
                     int32_t itemsize, int32_t path, int32_t lane_bytes,
                     int64_t work, int64_t row_bytes, void* stream);

/* Chained chunk GEMMs (blockwise matmul / tensordot with the k-sum fused):
 * task t computes C_t (=|+=) sum over its segments s of A_s @ B_s, row-major
 * views, every A_s m x k_s, every B_s k_s x n, accumulated in one continuous
 * K loop (f32 for f32/bf16 inputs, f64 / wrapping int64 otherwise) and
 * rounded to out_dtype once.  Replaces, per OUTPUT chunk, the (i, k, j)
 * tasks of _matmul (cubed/array_api/linear_algebra_functions.py:35-52,62-64:
 * one numpy BLAS call per chunk pair) together with the _sum_wo_cat
 * reduction over k (:52,67-78) that reads their partial products back; a
 * per-chunk product is a chain of one segment.  Host copies of both tables
 * (tasks, segs) are validated and pick the kernel; the device copies are
 * what the kernels read.  d_zero: >= 64 zero bytes of device memory (the
 * bf16 path reads k past the chain's end from it).  path: CUBED_GEMM_AUTO,
 * or CUBED_GEMM_ANY to force the element-wise kernel (tests). */
typedef struct {
  int64_t c;            /* output chunk base (device byte address)           */
  int64_t m, n, ldc;    /* output extents and row pitch (elements)           */
  int64_t seg0, nseg;   /* segments [seg0, seg0 + nseg) of the segment table  */
  int64_t ktot;         /* sum of the segments' k                            */
  int64_t accumulate;   /* 1: C += ..., 0: C = ...                           */
} cubed_gemm_chain_t;

typedef struct {
  int64_t a, b;         /* device byte addresses of A_s (m x k) and B_s (k x n) */
  int64_t k;            /* contracted extent of this pair                      */
  int64_t lda, ldb;     /* row pitches in elements                             */
  int64_t pad;
} cubed_gemm_seg_t;

#define CUBED_GEMM_AUTO (-1)
#define CUBED_GEMM_ANY 0   /* element-wise tiles, any dtype and shape          */
#define CUBED_GEMM_MFMA 1  /* bf16 (16x16x32) / f32 (32x32x2) MFMA tiles       */

/* Kernel the chain set would run on (CUBED_GEMM_MFMA or CUBED_GEMM_ANY). */
int cubed_gemm_chain_path(const cubed_gemm_chain_t* tasks, int64_t ntasks,
                          const cubed_gemm_seg_t* segs, int32_t in_dtype, int32_t out_dtype);
int cubed_gemm_chain(const cubed_gemm_chain_t* tasks, const cubed_gemm_chain_t* d_tasks,
                     int64_t ntasks, const cubed_gemm_seg_t* segs, const cubed_gemm_seg_t* d_segs,
                     int64_t nsegs, int32_t in_dtype, int32_t out_dtype, const void* d_zero,
                     int32_t path, void* stream);

/* Grid tiling (f32 / bf16 MFMA): the ti x tj tasks are the C-order chunk grid
 * of ONE (M, N) output (task I*tj + J = chunk (I, J); chunks cm x cn with cm,
 * cn >= 256 and cn % 4 (f32) / 8 (bf16) == 0 except the last row / column; every task the
 * same k segmentation).  256 x 256 tiles then cover the whole matrix --
 * a tile straddling chunk boundaries reads each row / column from its own
 * chunk -- instead of padding every chunk to whole tiles.  Same results
 * contract as cubed_gemm_chain (each element one f32 accumulation chain over
 * K in the same order).  cubed_gemm_grid_check (host only): 0 when the
 * tables fit, CUBED_E_LAYOUT (message set) otherwise. */
int cubed_gemm_grid_check(const cubed_gemm_chain_t* tasks, int64_t ti, int64_t tj,
                          const cubed_gemm_seg_t* segs, int64_t nsegs, int32_t in_dtype, int32_t out_dtype);
int cubed_gemm_chain_grid(const cubed_gemm_chain_t* tasks, const cubed_gemm_chain_t* d_tasks, int64_t ti,
                          int64_t tj, const cubed_gemm_seg_t* segs, const cubed_gemm_seg_t* d_segs,
                          int64_t nsegs, int32_t in_dtype, int32_t out_dtype, const void* d_zero,
                          void* stream);

/* Packed operands (bf16 in, f32 / bf16 out; f32 in, f32 out): the same chain
 * set as cubed_gemm_chain_grid, additionally ONE chunked product (segment s of
 * every task in chunk row I reads the same A chunk, in chunk column J the same
 * B chunk).  Both operands are first rewritten into the workspace as blocks
 * that are the GEMM's LDS image (bf16: 32 KiB per 256-row A panel / 256-column
 * B^T panel and 64-k tile; f32: 16 KiB per 256-row A panel / 256-column B
 * panel and 16-k step; K segments concatenated, pads zero), then one launch
 * tiles the whole output.  Same results contract as cubed_gemm_chain
 * (bit-identical to its MFMA paths).
 * cubed_gemm_pack_bytes (host only): workspace bytes the set needs, or a
 * negative CUBED_E_* with the message set when it does not pack.
 * cubed_gemm_chain_packed: d_ws 256-B aligned, ws_bytes >= that size
 * (else CUBED_E_WORKSPACE); stream-ordered, the workspace is free again once
 * the launches have run. */
int64_t cubed_gemm_pack_bytes(const cubed_gemm_chain_t* tasks, int64_t ti, int64_t tj,
                              const cubed_gemm_seg_t* segs, int64_t nsegs, int32_t in_dtype, int32_t out_dtype);
int cubed_gemm_chain_packed(const cubed_gemm_chain_t* tasks, const cubed_gemm_chain_t* d_tasks, int64_t ti,
                            int64_t tj, const cubed_gemm_seg_t* segs, const cubed_gemm_seg_t* d_segs,
                            int64_t nsegs, int32_t in_dtype, int32_t out_dtype, void* d_ws, int64_t ws_bytes,
                            void* stream);

/* Multi-GPU matmul on packed operands (ABI 15).  Replaces, on W ranks, the
 * same _matmul chunk products + _sum_wo_cat k-sum
 * (cubed/array_api/linear_algebra_functions.py:35-78) when the block-cyclic
 * ownership gives every k chunk of A one rank and every chunk column of C
 * (and of B) one rank.  A is packed into ONE k-major image of the whole A
 * (block (mt, kt) at (kt * TM + mt) * block bytes; bf16: 32 KiB blocks of 256
 * rows x 64 k, f32: 16 KiB of 256 rows x 16 k, the single-GPU packed blocks),
 * so the k blocks a rank packs are one contiguous byte run it sends whole to
 * every peer; the block straddling two k chunks is packed by the owner of
 * the first one from a received halo of the next chunk's first columns.
 * Every element stays the single-GPU packed path's f32 chain over K.
 * cubed_gemm_dist_image_bytes (host only): the image's size.
 * cubed_gemm_dist_pack_a: a_tasks = one task per A chunk row (m rows,
 *   segments = its k chunks: a = the chunk, a halo buffer (lda = its width)
 *   or 0 where the rank has neither); packs k blocks [kt0, kt1), which must
 *   read only present segments (else CUBED_E_LAYOUT, nothing launched).
 * cubed_gemm_dist_b_bytes / cubed_gemm_dist_pack_b: B (B^T for bf16) of the
 *   rank's own C chunk grid (ti x tj tasks, as cubed_gemm_chain_packed; the
 *   A addresses are not read) packed into d_ws.
 * cubed_gemm_dist_gemm: the rank's C chunks from the filled image and d_ws. */
int64_t cubed_gemm_dist_image_bytes(int64_t M, int64_t K, int32_t in_dtype);
int cubed_gemm_dist_pack_a(const cubed_gemm_chain_t* a_tasks, const cubed_gemm_chain_t* d_a_tasks, int64_t ti,
                           const cubed_gemm_seg_t* a_segs, const cubed_gemm_seg_t* d_a_segs, int64_t nsegs,
                           int32_t in_dtype, int64_t kt0, int64_t kt1, void* d_image, int64_t image_bytes,
                           void* stream);
int64_t cubed_gemm_dist_b_bytes(const cubed_gemm_chain_t* tasks, int64_t ti, int64_t tj,
                                const cubed_gemm_seg_t* segs, int64_t nsegs, int32_t in_dtype, int32_t out_dtype);
int cubed_gemm_dist_pack_b(const cubed_gemm_chain_t* tasks, const cubed_gemm_chain_t* d_tasks, int64_t ti,
                           int64_t tj, const cubed_gemm_seg_t* segs, const cubed_gemm_seg_t* d_segs, int64_t nsegs,
                           int32_t in_dtype, int32_t out_dtype, void* d_ws, int64_t ws_bytes, void* stream);
int cubed_gemm_dist_gemm(const cubed_gemm_chain_t* tasks, const cubed_gemm_chain_t* d_tasks, int64_t ti, int64_t tj,
                         const cubed_gemm_seg_t* segs, int64_t nsegs, int32_t in_dtype, int32_t out_dtype,
                         const void* d_image, int64_t image_bytes, const void* d_ws, int64_t ws_bytes,
                         void* stream);

/* ---- Zarr v2 chunk codecs (host only; cubed_amd/csrc/codec.cpp) --------
 * Replace numcodecs.Blosc's decode/encode behind zarr's chunk reads and
 * writes (storage/zarr.py:8-103 LazyZarrArray.create/open; the chunk I/O of
 * core/ops.py:88-182 from_zarr / store / to_zarr).  Reentrant, no GPU calls.
 * cubed_blosc_decompress: dst must hold exactly the frame's nbytes.
 * cubed_blosc_compress: lz4 + byte shuffle (shuffle != 0), unsplit blocks;
 * dst must hold cubed_blosc_max_compressed(nbytes); returns the frame size
 * or a negative error. */
int cubed_blosc_header(const void* src, int64_t srclen, int64_t* nbytes, int64_t* cbytes,
                       int* typesize, int* flags);
int cubed_blosc_decompress(const void* src, int64_t srclen, void* dst, int64_t dstlen);
int64_t cubed_blosc_max_compressed(int64_t nbytes);
/* Standalone numcodecs chunk codecs (zarr compressor ids "zstd" and "lz4"):
 * one zstd frame (decoded by the system libzstd, loaded on first use;
 * CUBED_E_UNSUPPORTED when it is absent) / a little-endian int32 size + one
 * LZ4 block.  dst must hold exactly the decoded size. */
int cubed_zstd_decompress(const void* src, int64_t srclen, void* dst, int64_t dstlen);
int cubed_lz4_chunk_decompress(const void* src, int64_t srclen, void* dst, int64_t dstlen);
int64_t cubed_blosc_compress(const void* src, int64_t nbytes, int typesize, int shuffle, void* dst,
                             int64_t dstcap);

/* library info */
int cubed_abi_version(void);
const char* cubed_last_error(void);
int cubed_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* CUBED_AMD_H */
