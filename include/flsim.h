/*
 * flsim.h -- C-ABI of libflsim.so, the MI355X (gfx950) engine for the federated-learning
 * simulation hot path of grossmanlev/FL-distributed-delay.
 *
 * The reference is pure Python; its "interface" for this path is the call sites below.  Each
 * entry point names the reference code it replaces.  All device pointers are raw HIP device
 * addresses (e.g. torch tensor data_ptr()), all work is enqueued on `stream` and is
 * asynchronous; no entry point allocates device memory or synchronises.  Status: 0 = OK,
 * 1 = invalid argument / the reference would raise, 2 = HIP error; flsim_last_error() gives the
 * message (thread-local).
 */
#ifndef FLSIM_H
#define FLSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* flsim_stream_t; /* == hipStream_t */

/* one simulated worker-step of a chunk: epoch t, worker i, dataset index k (main.py:138).
 * pad = the worker's batch size B (main.py:43-44 --batch_size; 0 = the default 128): a batch of
 * B samples spans ceil(B/128) consecutive records (128-sample groups) whose i is worker +
 * g * 2^20 for group g (the group's dropout key); sample slot j of group g is sample g*128 + j
 * of the worker's batch, drawn with the worker's key; slots past B are padding that adds no loss
 * and no gradient; the CrossEntropyLoss gradient is the mean over the B samples.  worker_loss of
 * a group = its summed loss / 128, so the worker's loss = sum over its groups * 128 / B. */
typedef struct WorkerRec {
    uint32_t t;
    uint32_t i;
    uint32_t k;
    uint32_t pad;
} WorkerRec;

const char* flsim_last_error(void);

/* ---------------------------------------------------------------------------------------------
 * The one collective of a sharded server step: each rank computes its contiguous
 * block of the epoch's workers (main.py:137-178 split across GPUs) into a partial
 * [S_t | losses]; one all-reduce (sum, fp32, in place) over RCCL / xGMI then gives every rank the
 * sum that rule() (main.py:184) and Adam (main.py:188) consume, replicated.  The reference has no
 * collective (one process, main.py:137); this is its replacement for a caller that does not use
 * torch.distributed.  RCCL is bound at run time: the copy already loaded in the process (e.g.
 * torch's), else $FLSIM_RCCL_LIB, else librccl.so.1.
 *   flsim_comm_unique_id: rank 0 makes the id (ncclGetUniqueId) and ships it to the others;
 *   flsim_comm_create(nranks, rank, id): ncclCommInitRank; nranks = 1 with id = NULL is a local
 *     communicator that never touches RCCL (its all-reduce is the identity);
 *   flsim_allreduce_sum: ncclAllReduce(buf, buf, count, float32, sum) on `stream`.
 * ------------------------------------------------------------------------------------------- */
#define FLSIM_COMM_ID_BYTES 128
typedef struct flsim_comm flsim_comm;
int flsim_comm_unique_id(unsigned char* id /* FLSIM_COMM_ID_BYTES */);
int flsim_comm_create(int nranks, int rank, const unsigned char* id, flsim_comm** out);
int flsim_comm_size(const flsim_comm* comm);
int flsim_comm_rank(const flsim_comm* comm);
int flsim_allreduce_sum(flsim_comm* comm, float* buf, size_t count, flsim_stream_t stream);
int flsim_comm_destroy(flsim_comm* comm);

/* ---------------------------------------------------------------------------------------------
 * Schedule (host): replaces the integer scan of main.py:119-123 (state), :150-166 (slow worker
 * + pesky_worker_grads FIFO), :167-178 (fast worker + throttle), :180-181 (window decrement).
 * delays[i] != 0 marks a slow worker (reference: only i = n-1, delay = --delay);
 * FLSIM_DELAY_ZERO marks the reference's slow worker under --delay 0: it computes and pushes at
 * t = 0 (main.py:153-157), and the epoch t = 1 fails like main.py:158's t % 0.
 * ------------------------------------------------------------------------------------------- */
#define FLSIM_DELAY_ZERO ((int32_t)0x80000000)
typedef struct flsim_sched flsim_sched;
flsim_sched* flsim_sched_create(int32_t n, const int32_t* delays, int32_t throttle,
                                int32_t max_throttle);
void flsim_sched_destroy(flsim_sched* s);
/* computes[n], fast[n]: u8 flags; stale_worker[n], stale_src[n]: popped FIFO entries in append
 * order; info[4] = {c_t, s_t, pushed, t}.  Returns 1 where main.py would raise IndexError in
 * rule() (empty weight_ups). */
int flsim_sched_epoch(flsim_sched* s, uint8_t* computes, uint8_t* fast, int32_t* stale_worker,
                      int64_t* stale_src, int64_t* info);
void flsim_sched_state(const flsim_sched* s, int64_t* out3);

/* ---------------------------------------------------------------------------------------------
 * PerformantNet1 worker-batched forward/backward: replaces Worker.fwd_bkwd (agents.py:32-40)
 * for every worker of a chunk at once, on models.py:11-47, including the batch draw of
 * main.py:138-142 (synthetic CIFAR-shaped u8 pool, ToTensor + Normalize via `lut`).
 * Gradients of all chunks of an epoch accumulate (agents.py:35 in-place .grad accumulation)
 * into split-K slabs inside `gradstate`; flsim_pn1_end_epoch sums them into S_t (torch
 * named_parameters layout, P = flsim_pn1_param_count() floats).
 * ------------------------------------------------------------------------------------------- */
long flsim_pn1_param_count(void);
long flsim_pn1_gradstate_bytes(void);
long flsim_pn1_workspace_bytes(int max_samples);
int flsim_pn1_workspace_offset(int which, int samples, long* offset_bytes);
/* (debug / tests) the tensors that feed the split-bf16 GEMMs are stored split (HM + L parts,
 * DESIGN 6g): the workspace id of tensor `which`'s L part, or -1 when it is stored fp32 */
int flsim_pn1_workspace_split_part(int which);
/* (debug / tests) 1 when workspace tensor `which` is stored channel-slice-major, [samples][C/16]
 * [H][W][16] (the inputs of conv2-4: a1, d1, a3), 0 when pixel-major [samples][H][W][C] */
int flsim_pn1_workspace_slice_major(int which);
/* packs theta_t into the kernel layouts and zeroes the slabs (start of main.py:126 epoch) */
int flsim_pn1_begin_epoch(void* gradstate, const float* theta, flsim_stream_t stream);
/* workers: device array of n_chunk_workers WorkerRec; worker_loss: device float per worker
 * (agents.py:40 lossval); backward_pass 0 = forward + loss only (eval / debugging) */
int flsim_pn1_fwd_bwd_chunk(void* gradstate, void* workspace, int max_samples, const float* theta,
                            const uint8_t* pool, const int32_t* labels, const int32_t* list_a,
                            int len_a, const int32_t* list_b, int len_b, const float* lut,
                            const WorkerRec* workers, int n_chunk_workers, int n_workers_total,
                            uint64_t seed, int dropout, int backward_pass, float* worker_loss,
                            flsim_stream_t stream);
/* pipelined variant of flsim_pn1_fwd_bwd_chunk (backward_pass always 1), the engine side of the
 * same main.py:137-178 worker loop: the batch draw, forward and loss run on `stream`, the
 * backward on the gradstate's own backward stream after this forward and after the previous
 * call's backward, so one chunk's forward overlaps the previous chunk's backward.  Successive
 * calls must alternate two workspaces (a forward waits for the backward that last used its
 * workspace).  Every other flsim_pn1_* entry point on the gradstate first makes `stream` wait
 * for the outstanding backward work, so end_epoch / server_step / begin_epoch see all chunks. */
int flsim_pn1_fwd_bwd_chunk_async(void* gradstate, void* workspace, int max_samples,
                                  const float* theta, const uint8_t* pool, const int32_t* labels,
                                  const int32_t* list_a, int len_a, const int32_t* list_b,
                                  int len_b, const float* lut, const WorkerRec* workers,
                                  int n_chunk_workers, int n_workers_total, uint64_t seed,
                                  int dropout, float* worker_loss, flsim_stream_t stream);
/* pipelined form of flsim_pn1_fwd_bwd_input (backward_pass always 1; the facade's
 * Worker.fwd_bkwd, agents.py:32-40): worker_loss is ready on `stream` after the forward, and the
 * backward overlaps the next call's forward.  Same workspace alternation and join rule as
 * flsim_pn1_fwd_bwd_chunk_async. */
int flsim_pn1_fwd_bwd_input_async(void* gradstate, void* workspace, int max_samples,
                                  const float* theta, const float* x, const int64_t* y,
                                  int n_samples, const WorkerRec* workers, uint64_t seed,
                                  int dropout, float* worker_loss, flsim_stream_t stream);
/* The facade's deferred backward: Worker.fwd_bkwd (agents.py:32-40) with the backward of up to
 * 16,384 samples of calls batched into one pass.  All calls of an epoch use theta_t
 * (main.py:154,159,169), so a call runs only its forward + CrossEntropyLoss now (the loss is what
 * agents.py:40 returns) into workspace rows [row0, row0 + ceil(n/128)*128); x, y, workers and
 * worker_loss as for flsim_pn1_fwd_bwd_input.  row0 is a multiple of 128; max_samples <= 16384. */
int flsim_pn1_fwd_rows(void* gradstate, void* workspace, int max_samples, int row0,
                       const float* theta, const float* x, const int64_t* y, int n_samples,
                       const WorkerRec* workers, uint64_t seed, int dropout, float* worker_loss,
                       flsim_stream_t stream);
/* The deferred forward of 128-sample calls: flsim_pn1_load_rows stages a call's batch (x, y as
 * for flsim_pn1_fwd_rows) into rows [row0, row0 + ceil(n/128)*128) and returns; later
 * flsim_pn1_fwd_loaded_rows runs the forward + CrossEntropyLoss of staged rows
 * [row0, row0 + n_rows) as one batched pass, each 128-row group one whole batch (workers[g] its
 * dropout key, worker_loss[g] its mean loss, bit-identical to flsim_pn1_fwd_rows on that batch). */
int flsim_pn1_load_rows(void* gradstate, void* workspace, int max_samples, int row0,
                        const float* x, const int64_t* y, int n_samples, flsim_stream_t stream);
int flsim_pn1_fwd_loaded_rows(void* gradstate, void* workspace, int max_samples, int row0,
                              int n_rows, const float* theta, const WorkerRec* workers,
                              uint64_t seed, int dropout, float* worker_loss,
                              flsim_stream_t stream);
/* ...then one backward over rows [0, n_rows) (the same theta and dropout flag as their forwards)
 * adds every call's gradient to the epoch's slabs (agents.py:35 accumulation).  It runs on the
 * gradstate's backward stream after everything queued on `stream`, so the next chunk's forwards
 * (into a second workspace) overlap it; every other flsim_pn1_* entry point joins it first, and a
 * flsim_pn1_fwd_rows into the same workspace waits for it. */
int flsim_pn1_bwd_rows(void* gradstate, void* workspace, int max_samples, int n_rows,
                       const float* theta, int dropout, flsim_stream_t stream);
/* explicit batch variant (Worker.fwd_bkwd(inp, outp), agents.py:32): x NCHW fp32 [n][3][32][32],
 * y int64 [n], any n >= 1 (main.py:43-44 --batch_size; at most 16384): padded to whole groups of
 * 128 samples that add nothing; the gradient is CrossEntropyLoss's mean over the n samples
 * (agents.py:34-35).  workers[ceil(n/128)] give each group's dropout RNG key; worker_loss[g] =
 * group g's summed loss / 128 (so the batch loss = sum_g worker_loss[g] * 128 / n). */
int flsim_pn1_fwd_bwd_input(void* gradstate, void* workspace, int max_samples, const float* theta,
                            const float* x, const int64_t* y, int n_samples,
                            const WorkerRec* workers, uint64_t seed, int dropout,
                            int backward_pass, float* worker_loss, flsim_stream_t stream);
int flsim_pn1_end_epoch(void* gradstate, float* grad_out, flsim_stream_t stream);
/* the gradstate's buffer is about to be freed: drop the library's per-gradstate bookkeeping (the
 * slab rows written this epoch).  A backward pass on a gradstate with no flsim_pn1_begin_epoch
 * since creation or release fails with status 1. */
void flsim_pn1_release(void* gradstate);
/* eval of an explicit batch (util.py:31-45 print_test_accuracy's model(images), dropout off):
 * x NCHW fp32 [n_images][3][32][32] -> pred (device int32[n_images]) */
int flsim_pn1_eval_input(void* gradstate, void* workspace, int max_samples, const float* theta,
                         const float* x, int n_images, int32_t* pred, flsim_stream_t stream);
/* Evaluation: replaces util.print_test_accuracy (util.py:31-45) as called at main.py:196-210
 * after central.model.eval() (main.py:190: dropout off).  Forward of pool images
 * [first, first + n_images) (u8 NCHW 3x32x32, normalised through `lut`), predictions = argmax of
 * the logits (torch.max(outputs, 1): first maximum wins) into pred (device int32[n_images]).
 * Uses the gradstate's packed-weight area (re-packed from theta). */
int flsim_pn1_eval_pool(void* gradstate, void* workspace, int max_samples, const float* theta,
                        const uint8_t* pool, int first, int n_images, const float* lut,
                        int32_t* pred, flsim_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * VGG-11 worker-batched forward/backward (configs[4]'s larger CNN): replaces Worker.fwd_bkwd
 * (agents.py:32-40) when the central model is models.py:101-103 vgg11() (cfg 'A': 8 conv3x3
 * padding 1 + ReLU, 5 max-pools; classifier Dropout / Linear / ReLU twice + Linear,
 * models.py:50-98).  Same contract, argument meaning and errors as the flsim_pn1_* entry points
 * above; parameters flat in vgg11().named_parameters() order, P = flsim_vgg11_param_count()
 * = 9,750,922.  The classifier's dropouts use RNG sites 6 and 7 of the Philox spec.
 * ------------------------------------------------------------------------------------------- */
long flsim_vgg11_param_count(void);
long flsim_vgg11_gradstate_bytes(void);
long flsim_vgg11_workspace_bytes(int max_samples);
int flsim_vgg11_workspace_offset(int which, int samples, long* offset_bytes);
int flsim_vgg11_begin_epoch(void* gradstate, const float* theta, flsim_stream_t stream);
int flsim_vgg11_fwd_bwd_chunk(void* gradstate, void* workspace, int max_samples,
                              const float* theta, const uint8_t* pool, const int32_t* labels,
                              const int32_t* list_a, int len_a, const int32_t* list_b, int len_b,
                              const float* lut, const WorkerRec* workers, int n_chunk_workers,
                              int n_workers_total, uint64_t seed, int dropout, int backward_pass,
                              float* worker_loss, flsim_stream_t stream);
int flsim_vgg11_fwd_bwd_input(void* gradstate, void* workspace, int max_samples,
                              const float* theta, const float* x, const int64_t* y, int n_samples,
                              const WorkerRec* workers, uint64_t seed, int dropout,
                              int backward_pass, float* worker_loss, flsim_stream_t stream);
/* the facade's deferred fwd_bkwd for vgg11() (128-sample calls, agents.py:32-40): load_rows stages
 * a call's batch into workspace rows [row0, row0 + 128) as flsim_pn1_load_rows does; then
 * fwd_bwd_loaded_rows runs forward, CrossEntropyLoss and backward of the staged rows [0, n_rows) as
 * one batched chunk into the epoch's slabs (workers[g] / worker_loss[g]: one per 128-row call). */
int flsim_vgg11_load_rows(void* gradstate, void* workspace, int max_samples, int row0,
                          const float* x, const int64_t* y, int n_samples, flsim_stream_t stream);
int flsim_vgg11_fwd_bwd_loaded_rows(void* gradstate, void* workspace, int max_samples, int n_rows,
                                    const float* theta, const WorkerRec* workers, uint64_t seed,
                                    int dropout, float* worker_loss, flsim_stream_t stream);
/* vgg11_bn: the same two calls; each staged 128-row call is one BatchNorm batch, and bn_stats
 * [n_rows / 128][flsim_vgg11_bn_stats_per_worker()] receives the calls' statistics for
 * flsim_vgg11_bn_update_running (in call order, as nn.BatchNorm2d's per-call updates). */
int flsim_vgg11_bn_load_rows(void* gradstate, void* workspace, int max_samples, int row0,
                             const float* x, const int64_t* y, int n_samples,
                             flsim_stream_t stream);
int flsim_vgg11_bn_fwd_bwd_loaded_rows(void* gradstate, void* workspace, int max_samples,
                                       int n_rows, const float* theta, const WorkerRec* workers,
                                       uint64_t seed, int dropout, float* worker_loss,
                                       float* bn_stats, flsim_stream_t stream);
int flsim_vgg11_end_epoch(void* gradstate, float* grad_out, flsim_stream_t stream);
int flsim_vgg11_eval_input(void* gradstate, void* workspace, int max_samples, const float* theta,
                           const float* x, int n_images, int32_t* pred, flsim_stream_t stream);
int flsim_vgg11_eval_pool(void* gradstate, void* workspace, int max_samples, const float* theta,
                          const uint8_t* pool, int first, int n_images, const float* lut,
                          int32_t* pred, flsim_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * VGG-11 with BatchNorm (models.py:106-108 vgg11_bn(): Conv2d -> BatchNorm2d -> ReLU per conv,
 * models.py:88-89): replaces Worker.fwd_bkwd (agents.py:32-40) when the central model is
 * vgg11_bn().  Same contract as flsim_vgg11_*; parameters flat in vgg11_bn().named_parameters()
 * order (conv weight, conv bias, BatchNorm weight, BatchNorm bias per layer), P = 9,756,426.
 * Train mode: every simulated worker's 128 samples are one BatchNorm batch (one fwd_bkwd call);
 * bn_stats (device float[n_chunk_workers][flsim_vgg11_bn_stats_per_worker()] or nullptr)
 * receives each worker's per-layer [batch mean | unbiased batch variance], the inputs of the
 * running-buffer update nn.BatchNorm2d does on every call.  The running buffers are a device
 * float[5504]: [running_mean | running_var] of features.1, .5, .9, .12, .16, .19, .23, .26.
 * ------------------------------------------------------------------------------------------- */
long flsim_vgg11_bn_param_count(void);
long flsim_vgg11_bn_gradstate_bytes(void);
long flsim_vgg11_bn_workspace_bytes(int max_samples);
int flsim_vgg11_bn_workspace_offset(int which, int samples, long* offset_bytes);
int flsim_vgg11_bn_stats_per_worker(void);
int flsim_vgg11_bn_begin_epoch(void* gradstate, const float* theta, flsim_stream_t stream);
int flsim_vgg11_bn_fwd_bwd_chunk(void* gradstate, void* workspace, int max_samples,
                                 const float* theta, const uint8_t* pool, const int32_t* labels,
                                 const int32_t* list_a, int len_a, const int32_t* list_b,
                                 int len_b, const float* lut, const WorkerRec* workers,
                                 int n_chunk_workers, int n_workers_total, uint64_t seed,
                                 int dropout, int backward_pass, float* worker_loss,
                                 float* bn_stats, flsim_stream_t stream);
int flsim_vgg11_bn_fwd_bwd_input(void* gradstate, void* workspace, int max_samples,
                                 const float* theta, const float* x, const int64_t* y,
                                 int n_samples, const WorkerRec* workers, uint64_t seed,
                                 int dropout, int backward_pass, float* worker_loss,
                                 float* bn_stats, flsim_stream_t stream);
int flsim_vgg11_bn_end_epoch(void* gradstate, float* grad_out, flsim_stream_t stream);
/* vgg11_bn: explicit batches must be whole 128-sample groups (one BatchNorm batch each) */
int flsim_vgg11_bn_eval_input(void* gradstate, void* workspace, int max_samples,
                              const float* theta, const float* x, int n_images,
                              const float* running, int32_t* pred, flsim_stream_t stream);
/* util.py:31-45 in eval mode: BatchNorm normalises with the running buffers `running`. */
int flsim_vgg11_bn_eval_pool(void* gradstate, void* workspace, int max_samples,
                             const float* theta, const uint8_t* pool, int first, int n_images,
                             const float* lut, const float* running, int32_t* pred,
                             flsim_stream_t stream);
/* nn.BatchNorm2d's running update (momentum 0.1) for n_workers calls in worker order:
 * r = 0.1 * stat + 0.9 * r per call, stat from bn_stats[w] (w = 0 .. n_workers-1). */
int flsim_vgg11_bn_update_running(float* running, const float* bn_stats, int n_workers,
                                  flsim_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Server step: replaces Agg.rule = rule() (main.py:23-25, agents.py:43-45: per-tensor
 * torch.stack(weight_ups).mean(0)) + Central.update_model (agents.py:9-21: Adam step,
 * main.py:106).  Bit-exact with torch 2.10 CPU except sqrt rounding;
 * step = Adam step count after increment.
 *
 * flsim_rule describes weight_ups: the entries are S_t (every fast worker's aliased .grad,
 * main.py:172) or one of `arrays` (popped stale FIFO entries, main.py:161-165; NULL = zeros, the
 * torch-1.x semantics).
 *   prog == NULL : reference order, [S_t] * c followed by arrays[0 .. n_arrays) (the slow worker
 *                  is the last worker, main.py:150);
 *   prog != NULL : general order (heterogeneous-delay extension, SURVEY 8 a1: entries appended in
 *                  worker-index order): a device program from flsim_cascade_program, info = its
 *                  info words.
 * k is the divisor of the mean (= the entry count, main.py:24; the independent-entry semantics
 * passes S = the sum of k distinct entries with c = 1).
 * ------------------------------------------------------------------------------------------- */
#define FLSIM_MAX_ARRAYS 64
typedef struct flsim_rule {
    int32_t k;
    int32_t c;
    const int32_t* prog;
    int32_t info[4];
    int32_t n_arrays;
    const float* arrays[FLSIM_MAX_ARRAYS];
} flsim_rule;

/* host: the summation program of rule() over k entries whose non-S_t entries sit at positions
 * pos[0 .. n_events) (increasing) and hold arrays arr[] (indices into flsim_rule.arrays; at most
 * 64), in the device's macro-word form: prog[0 .. cap) receives (lo, hi) int32 pairs plus one
 * padding pair; info[4] = {pairs, pair index of the row_sum part, flags, level power}.
 * k <= 524288. */
int flsim_cascade_program(int k, const int32_t* pos, const int32_t* arr, int n_events,
                          int32_t* prog, int cap, int32_t* info);
/* host (testing): run a macro program on the host, out[e] = cascade sum for element e (x = S[e],
 * entry arrays ys[q][e]; tail[e] != 0 selects the row_sum part) */
int flsim_cascade_eval_host(const int32_t* prog, const int32_t* info, const float* S,
                            const float* const* ys, int n_arrays, const uint8_t* tail, long n,
                            float* out);

/* rule() + Adam from S_t in a buffer (world > 1 after the all-reduce; the FL.agents facade).
 * tensor_sizes: numel of each parameter tensor in named_parameters order (the cascade's column
 * rule is per tensor). */
int flsim_aggregate_adam_rule(const float* S, const flsim_rule* rule, float* p, float* m, float* v,
                              long P, const long* tensor_sizes, int n_tensors, long step, double lr,
                              double beta1, double beta2, double eps, flsim_stream_t stream);
/* the same, also writing S_t into S_out (nullable; 16-byte aligned) in the same pass: the slow
 * worker's FIFO entry at a tick (main.py:156,161) when S_t arrives in a buffer (world > 1, after
 * the all-reduce) */
int flsim_aggregate_adam_rule_push(const float* S, float* S_out, const flsim_rule* rule, float* p,
                                   float* m, float* v, long P, const long* tensor_sizes,
                                   int n_tensors, long step, double lr, double beta1, double beta2,
                                   double eps, flsim_stream_t stream);
/* convenience forms of the above: reference order with n_stale <= 8 stale entries; and the
 * independent-entry semantics (S = sum of k distinct entries, mean = S / k) */
int flsim_aggregate_adam(const float* S, int c, const float* const* stale, int n_stale,
                         float* p, float* m, float* v, long P, const long* tensor_sizes,
                         int n_tensors, long step, double lr, double beta1, double beta2,
                         double eps, flsim_stream_t stream);
int flsim_aggregate_adam_sum(const float* S, int k, float* p, float* m, float* v, long P,
                             const long* tensor_sizes, int n_tensors, long step, double lr,
                             double beta1, double beta2, double eps, flsim_stream_t stream);

/* Fused end of an epoch at world = 1: S_t = sum of the gradstate's slabs (what
 * flsim_<net>_end_epoch computes), written to S_out if non-NULL (the slow worker's FIFO entry at a
 * tick, main.py:156,161), then rule() + Adam -- one launch, S_t never round-trips through HBM. */
int flsim_pn1_server_step(void* gradstate, float* S_out, const flsim_rule* rule, float* p,
                          float* m, float* v, long step, double lr, double beta1, double beta2,
                          double eps, flsim_stream_t stream);
int flsim_vgg11_server_step(void* gradstate, float* S_out, const flsim_rule* rule, float* p,
                            float* m, float* v, long step, double lr, double beta1, double beta2,
                            double eps, flsim_stream_t stream);
int flsim_vgg11_bn_server_step(void* gradstate, float* S_out, const flsim_rule* rule, float* p,
                               float* m, float* v, long step, double lr, double beta1,
                               double beta2, double eps, flsim_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Measurement (no reference counterpart): HIP events around every worker-batched GEMM launch on
 * its stream, for bench.py's live roofline figure.  read() fills flsim_probe_kernel_count()
 * entries per kernel id (launches, total ms, total algorithmic FLOPs) and resets the record.
 * ------------------------------------------------------------------------------------------- */
int flsim_probe_enable(int capacity);
int flsim_probe_read(int* launches, double* total_ms, double* total_flops);
int flsim_probe_disable(void);
int flsim_probe_kernel_count(void);
const char* flsim_probe_kernel_name(int kid);

#ifdef __cplusplus
}
#endif

#endif /* FLSIM_H */
