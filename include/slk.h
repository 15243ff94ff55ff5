/*
 * slk.h — C-ABI of the MI355X-native split-CNN step (libslk.so, gfx950).
 *
 * The reference (eliasandronicou/split-learning-k8s) has no native code and no FFI: every op of its
 * hot path is a torch CPU call made by src/model_def.py, src/client_part.py and src/server_part.py.
 * Each entry point below replaces one (or a fused group) of those calls; the reference call site is
 * cited next to each declaration. The Python host layer (split-learning-k8s_amd/splitcnn/_lib.py)
 * binds these with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions (all entry points):
 *   - Plain pointers to DEVICE memory, sizes as int, the HIP stream as `void*` (hipStream_t).
 *   - Every buffer, including workspaces, is allocated by the caller. The library never allocates,
 *     frees or synchronises, so every call is safe inside HIP-graph capture.
 *   - Return value: 0 on success, otherwise a hipError_t code (1 = hipErrorInvalidValue for bad
 *     arguments). slk_error_string() turns it into text. Nothing throws across the ABI.
 *   - Stateless and reentrant; ordering comes only from the caller's stream.
 *   - Layouts are the reference's logical NCHW layouts (torch contiguous):
 *       x      f32 [B,1,28,28]      client input           (client_part.py:110,114)
 *       act    f32 [B,32,26,26]     cut-layer activations  (client_part.py:114,118)
 *       pooled f32 [B,64,12,12]     = flatten [B,9216], index c*144+h*12+w (model_def.py:20-21,26-27)
 *       code   u8  [B,64,12,12]     max-pool argmax in its 2x2 window, row-major 0..3, first max wins;
 *                                   4 = pooled value <= 0 (ReLU blocks the gradient)
 *       logits f32 [B,10]; labels i64 [B]
 *       W1 f32[32,1,3,3] b1[32]  W2 f32[64,32,3,3] b2[64]  W3 f32[10,9216] b3[10]  (model_def.py:8,18,22)
 *   - Flat parameter blocks (what the fused SGD updates in one launch):
 *       client: [W1 (288) | b1 (32)]                     = SLK_CLIENT_NPARAM floats
 *       server: [W2 (18432) | b2 (64) | W3 (92160) | b3 (10)] = SLK_SERVER_NPARAM floats
 *   - Tensors, parameters, accumulators and every non-conv2 kernel are fp32 (the reference's dtype).
 *     conv2's products come in two forms: the f32 MFMA (Winograd slk_conv2_*, direct slk_conv2_*_direct)
 *     and "x3" (slk_conv2_*_x3*, the default fused step's): each f32 operand is scaled by an exact power
 *     of two and split into f16 hi + lo, and a product is hi*hi + hi*lo + lo*hi on the f16 MFMA with
 *     f32 accumulation (per-product error <= ~7e-7 relative; tested against fp64 at the f32 path's bars).
 *     Weight-gradient reductions use per-workgroup slabs summed in a fixed order, so every result is
 *     run-to-run bit-stable.
 */
#ifndef SLK_H
#define SLK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLK_ABI_VERSION 1

#define SLK_CLIENT_NPARAM 320
#define SLK_SERVER_NPARAM 110666
#define SLK_OFF_W2 0
#define SLK_OFF_B2 18432
#define SLK_OFF_W3 18496
#define SLK_OFF_B3 110656

int slk_abi_version(void);
const char* slk_error_string(int err);
/* Hex sha256 of the sources this library was compiled from (the csrc .hip and .h files, include/slk.h);
 * splitcnn/_lib.py refuses a library whose id differs from the tree's. */
const char* slk_build_id(void);

/* ---------------------------------------------------------------- client stage (ModelPartA) */

/* act = relu(conv2d(x, W1, b1)), stride 1, no padding.
 * Replaces ModelPartA.forward (src/model_def.py:11-12) as called at src/client_part.py:114. */
int slk_conv1_fwd(const float* x, const float* W1, const float* b1, float* act, int B, void* stream);

/* slk_conv1_fwd that also writes act_amax[b], the per-sample scale value of the x3 conv2 kernels: since
 * round 5 the bound max_c (sum_k |W1[c][k]| * max|x[b]| + max(b1[c], 0)) >= max(act[b]) (one float expression,
 * slk_common.h conv1_cut_bound; the same value slk_conv1_fwd_x3 emits), so the 354 MB cut is never re-read
 * and no writer needs a pass over its outputs before splitting them. */
int slk_conv1_fwd_amax(const float* x, const float* W1, const float* b1, float* act, float* act_amax, int B,
                       void* stream);

/* Client backward: relu-bwd mask (act > 0) applied to the cut gradient, then conv1 weight/bias
 * gradient. No input gradient (the data needs none). Writes per-group partial slabs
 * [slk_conv1_wgrad_nslab(B)][320] into `slabs`; reduce them with slk_sgd_from_slabs or
 * slk_reduce_slabs. Replaces `activations.backward(server_grads)` (src/client_part.py:132). */
int slk_conv1_wgrad(const float* x, const float* act, const float* cut_grad, float* slabs, int B,
                    void* stream);
int slk_conv1_wgrad_nslab(int B);
/* Same result as slk_conv1_wgrad, with the ReLU mask recomputed from x, W1, b1 in slk_conv1_fwd's
 * exact FMA order (act > 0 <=> conv1(x) > 0, bit-identically) instead of read from `act`: 89.6 KB of
 * HBM traffic per sample instead of 176 KB. W1/b1 must be the forward's weights (they are inside a
 * split step: the client's SGD follows its backward, client_part.py:132-133). */
int slk_conv1_wgrad_remask(const float* x, const float* W1, const float* b1, const float* cut_grad, float* slabs,
                           int B, void* stream);

/* ---------------------------------------------------------------- server stage (ModelPartB) */

/* pooled = maxpool2(relu(conv2d(act, W2, b2))) and its argmax code, fused (Winograd F(2x2,3x3) on
 * the f32 MFMA: one transformed 2x2 output tile = one pool window). Replaces ModelPartB.forward lines
 * src/model_def.py:25-27 as called at src/server_part.py:48. */
int slk_conv2_fwd_pool(const float* act, const float* W2, const float* b2, float* pooled,
                       uint8_t* code, int B, void* stream);
/* The same op as a direct implicit GEMM (f32 MFMA, k-ordered fma chains); kept as the A/B and
 * cross-check path. */
int slk_conv2_fwd_pool_direct(const float* act, const float* W2, const float* b2, float* pooled,
                              uint8_t* code, int B, void* stream);

/* logits = pooled @ W3^T + b3.  Replaces model_def.py:28 (fc1). */
int slk_fc_fwd(const float* pooled, const float* W3, const float* b3, float* logits, int B,
               void* stream);

/* Cross-entropy (mean reduction, no label smoothing) forward+backward from logits:
 * loss_i[b] = logsumexp(z_b) - z_b[y_b];  dlogits = (softmax(z) - onehot(y)) * grad_scale.
 * grad_scale = 1/B reproduces nn.CrossEntropyLoss()'s mean (src/server_part.py:16,49,51).
 * An out-of-range label writes NaN loss/dlogits for that row and sets *err_flag (may be NULL). */
int slk_xent_fwd_bwd(const float* logits, const int64_t* labels, float* loss_i, float* dlogits,
                     float grad_scale, int* err_flag, int B, void* stream);

/* slk_fc_fwd + slk_xent_fwd_bwd in one launch (the cross-entropy of a workgroup's 16 samples from the logits it
 * just reduced, in LDS): the same logits, loss_i and dlogits bit for bit. src/server_part.py:48-49 + the CE part
 * of :51. */
int slk_fc_logits_xent(const float* pooled, const float* W3, const float* b3, const int64_t* labels, float* logits,
                       float* loss_i, float* dlogits, float grad_scale, int* err_flag, int B, void* stream);

/* dpooled = dlogits @ W3 (fc1 input gradient). Replaces the fc1 part of loss.backward()
 * (src/server_part.py:51). */
int slk_fc_dgrad(const float* dlogits, const float* W3, float* dpooled, int B, void* stream);
/* slk_fc_dgrad that also writes dp_amax[b] = max |dpooled[b]|: the split head of the x3 step (logits,
 * cross-entropy, fc1 weight gradient while pooled is still in the Infinity Cache, then this). */
int slk_fc_dgrad_amax(const float* dlogits, const float* W3, float* dpooled, float* dp_amax, int B, void* stream);

/* Fused server head: fc1 forward, cross-entropy forward+backward and fc1 input gradient in one
 * launch (pooled is read from HBM once for the logits and once, L2-hot, for nothing else).
 * Outputs logits, loss_i, dlogits, dpooled. Replaces server_part.py:48(fc1 part),49,51(fc1 part). */
int slk_fc_xent(const float* pooled, const float* W3, const float* b3, const int64_t* labels,
                float* logits, float* loss_i, float* dlogits, float* dpooled, float grad_scale,
                int* err_flag, int B, void* stream);

/* slk_fc_xent that also writes dp_amax[b] = max |dpooled[b]| (the x3 conv2 backward kernels' scales). */
int slk_fc_xent_amax(const float* pooled, const float* W3, const float* b3, const int64_t* labels, float* logits,
                     float* loss_i, float* dlogits, float* dpooled, float* dp_amax, float grad_scale, int* err_flag,
                     int B, void* stream);

/* fc1 weight/bias gradient partials: slabs [slk_fc_wgrad_nslab(B)][92170] laid out as
 * [dW3 (10*9216) | db3 (10)], i.e. the tail of the server flat block. */
int slk_fc_wgrad(const float* dlogits, const float* pooled, float* slabs, int B, void* stream);
int slk_fc_wgrad_nslab(int B);

/* Cut-layer gradient: cut_grad = conv2 input gradient of maxpool/relu-masked dpooled
 * (uses `code` from slk_conv2_fwd_pool). This is `client_activations.grad` of
 * src/server_part.py:45,51,57. Winograd F(2x2,3x3) on the f32 MFMA; the routed conv2 output
 * gradient is expanded per transform tile in registers (never materialised). */
int slk_conv2_dgrad(const float* dpooled, const uint8_t* code, const float* W2, float* cut_grad,
                    int B, void* stream);
/* The same op as a direct implicit GEMM (A/B and cross-check path). */
int slk_conv2_dgrad_direct(const float* dpooled, const uint8_t* code, const float* W2, float* cut_grad,
                           int B, void* stream);

/* conv2 weight/bias gradient partials: slabs [slk_conv2_wgrad_nslab(B)][18496] laid out as
 * [dW2 (64*288) | db2 (64)], i.e. the head of the server flat block; their fixed-order sum is the
 * gradient. Winograd F(2x2,3x3) filter gradient on the f32 MFMA (G^T dU G applied per slab). */
int slk_conv2_wgrad(const float* act, const float* dpooled, const uint8_t* code, float* slabs,
                    int B, void* stream);
int slk_conv2_wgrad_nslab(int B);
/* The same op as a direct implicit GEMM (A/B and cross-check path), with its own slab count. */
int slk_conv2_wgrad_direct(const float* act, const float* dpooled, const uint8_t* code, float* slabs,
                           int B, void* stream);
int slk_conv2_wgrad_direct_nslab(int B);

/* ---------------------------------------------------------------- conv2 on the f16 MFMA, fp32-grade ("x3")
 * The same ops as slk_conv2_fwd_pool / _dgrad / _wgrad, computed as direct implicit GEMMs whose f32
 * operands are split after an exact power-of-two scale into f16 hi + lo, each product formed by three
 * v_mfma_f32_16x16x32_f16 (hi*hi + hi*lo + lo*hi) into an f32 accumulator: per-product relative error
 * <= ~7e-7 (csrc/slk_x3.hip). Operand scales: weights per launch (from max|W2|), data per sample from a
 * caller-supplied per-sample max |.| (slk_row_amax, or a producer that emits it); the arrays must bound
 * their rows (a too-small bound overflows f16 to inf). Replace the same reference lines as the f32 ops. */

/* amax[r] = max_i |x[r*n + i]| for r < rows (NaNs ignored). */
int slk_row_amax(const float* x, int rows, int n, float* amax, void* stream);
/* slk_conv2_fwd_pool on the x3 path; act_amax[B] = per-sample max |act| (model_def.py:25-27). */
int slk_conv2_fwd_pool_x3(const float* act, const float* act_amax, const float* W2, const float* b2, float* pooled,
                          uint8_t* code, int B, void* stream);
/* slk_conv2_dgrad on the x3 path; dp_amax[B] = per-sample max |dpooled| (server_part.py:45,51,57). */
int slk_conv2_dgrad_x3(const float* dpooled, const float* dp_amax, const uint8_t* code, const float* W2,
                       float* cut_grad, int B, void* stream);
/* slk_conv2_wgrad on the x3 path: slabs [slk_conv2_wgrad_x3_nslab(B)][18496] = [dW2 | db2] partials
 * (fixed-order sum = the gradient). The reduction spans samples (server_part.py:51), so every product
 * carries one scale: the input keeps its sample's scale (from act_amax) and that sample's dY is scaled
 * to compensate (launch maxima of act_amax / dp_amax); db2 is summed in f32. */
int slk_conv2_wgrad_x3(const float* act, const float* act_amax, const float* dpooled, const float* dp_amax,
                       const uint8_t* code, float* slabs, int B, void* stream);
int slk_conv2_wgrad_x3_nslab(int B);
/* The forward that also writes its split f16 input images (act16, slk_conv2_act16_bytes(B) bytes; each
 * sample at its own scale from act_amax) and the wgrad that moves them by LDS-DMA instead of loading and
 * splitting act: the wgrad's input staging becomes a copy. Same results as slk_conv2_wgrad_x3 (bitwise:
 * the same scales, the same f16 values). */
int slk_conv2_fwd_pool_x3s(const float* act, const float* act_amax, const float* W2, const float* b2, float* pooled,
                           uint8_t* code, uint16_t* act16, int B, void* stream);
int slk_conv2_wgrad_x3s(const uint16_t* act16, const float* act_amax, const float* dpooled, const float* dp_amax,
                        const uint8_t* code, float* slabs, int B, void* stream);
/* Which kernel slk_conv2_wgrad_x3s runs (round 6): 2 = on the 2:4-sparse f16 MFMA (v_smfmac_f32_16x16x64_f16:
 * the max-pool routing leaves at most 2 nonzeros of dY in every 4 consecutive output pixels of a row starting at
 * a multiple of 4, so half the dense x3 products are never issued), 1 = the dense x3 kernel, 0 = the round-4
 * kernel. Measurement only (bench.py prices the executed products against the matching peak). */
int slk_conv2_wgrad_x3_form(void);
/* slk_conv2_fwd_pool_x3s with the per-sample max |act| computed inside the forward (written to act_amax,
 * the values slk_row_amax gives) instead of read: the drop-in module path has no separate pass over the cut.
 * act 16-byte aligned. Replaces the row_amax + forward pair behind ModelPartB.forward (src/model_def.py:25-26). */
/* Measurement only: the device's sustained dense f16 MFMA rate (v_mfma_f32_16x16x32_f16, 6 independent chains
 * per wave, 2 waves per SIMD, varied operands). out: slk_mfma_probe_blocks() * 256 floats; FLOPs per launch =
 * slk_mfma_probe_blocks() * 4 * iters * 6 * 16384. bench.py prices the kernels against it beside the nominal peak. */
int slk_mfma_probe_blocks(void);
int slk_mfma_probe(float* out, int iters, void* stream);
int slk_conv2_fwd_pool_x3sa(const float* act, float* act_amax, const float* W2, const float* b2, float* pooled,
                            uint8_t* code, uint16_t* act16, int B, void* stream);
/* act16 layout: per sample an h plane then an l plane, each [26 x 26 pixels][32 ci] f16 with 64-B pixels
 * (8-channel chunk c8 at slot c8 ^ (x & 2)): B x 86,528 bytes. */
int64_t slk_conv2_act16_bytes(int B);

/* The client's conv1 + ReLU (replaces slk_conv1_fwd_amax inside a fused step, src/client_part.py:114)
 * writing the x3 server operand directly: act_amax (the bound of slk_conv1_fwd_amax) and the act16 images
 * (bit-identical to those slk_conv2_fwd_pool_x3s writes from the f32 act with that act_amax), plus the f32
 * act when act != NULL — one pass per (pixel, 8-channel) item. The server forward then reads the
 * images (slk_conv2_fwd_pool_x3i: same pooled / code as slk_conv2_fwd_pool_x3 on the f32 act, bitwise)
 * and so does the wgrad (slk_conv2_wgrad_x3s). relu_bits (optional, slk_relu_bits_bytes(B) bytes, 16-byte
 * aligned): the ReLU mask act > 0 of every cut element, 1 bit each (per sample [4 channel groups cg][169]
 * u32, bit 4 (c & 7) + u of word (c >> 3, t) = act[c][4 t + u] > 0), which slk_conv2_dgrad_x3_c1w consumes. */
int slk_conv1_fwd_x3(const float* x, const float* W1, const float* b1, float* act, float* act_amax, uint16_t* act16,
                     uint32_t* relu_bits, int B, void* stream);
int64_t slk_relu_bits_bytes(int B);
int slk_conv2_fwd_pool_x3i(const uint16_t* act16, const float* act_amax, const float* W2, const float* b2,
                           float* pooled, uint8_t* code, int B, void* stream);

/* The x3 dgrad with the client's backward fused (src/server_part.py:51 -> src/client_part.py:132 in one
 * launch, for the single-GPU step): the cut gradient is not written; each workgroup applies the client's
 * ReLU mask (relu_bits from slk_conv1_fwd_x3) and writes one slab [dW1 c*9+tap (288) | db1 c (32)] of the
 * client gradient (slk_conv2_dgrad_x3_c1w_nslab(B) slabs, reduced by slk_sgd_from_slabs). */
int slk_conv2_dgrad_x3_c1w(const float* dpooled, const float* dp_amax, const uint8_t* code, const float* W2,
                           const float* x, const uint32_t* relu_bits, float* client_slabs, int B, void* stream);
int slk_conv2_dgrad_x3_c1w_nslab(int B);

/* ---------------------------------------------------------------- reductions / optimizer */

/* out[i] = (accumulate ? out[i] : 0) + sum_{s=0}^{nslab-1} slabs[s*n + i]  (fixed slab order).
 * accumulate = 1 sums micro-batches into one gradient (pipeline topologies).
 * Summation order (this and SGD from slabs): nslab <= 16 -> slabs in ascending order per column;
 * 16 < nslab <= 64 -> 4 partial sums over slabs w, w+4, w+8, ... (w = 0..3) added in w order; nslab > 64 ->
 * 16 partial sums over slabs w, w+16, ... added in w order (Adam from slabs: the same three forms). Each is
 * a fixed function of (slabs, nslab): bit-stable run to run, but results from different forms are not
 * bitwise comparable. */
int slk_reduce_slabs(const float* slabs, int nslab, int n, float* out, int accumulate, void* stream);

/* Fused deterministic slab reduction + SGD (lr, no momentum, no weight decay):
 * g = sum_s slabs[s*n+i]; grad[i] = g (if grad != NULL); param[i] -= lr * g.
 * Replaces optimizer.step() of optim.SGD(lr=0.01) (client_part.py:17,133; server_part.py:15,52). */
int slk_sgd_from_slabs(float* param, float* grad, const float* slabs, int nslab, int n, float lr,
                       void* stream);

/* param[i] -= lr * grad[i]  (flat multi-tensor SGD; torch.optim.SGD semantics, momentum 0). */
int slk_sgd(float* param, const float* grad, int n, float lr, void* stream);

/* out[0] = scale * sum(values[0..n))  (fixed-order reduction). With values = per-sample losses and
 * scale = 1/B this is nn.CrossEntropyLoss()'s mean (src/server_part.py:49). */
int slk_loss_sum(const float* values, int n, float scale, float* out, void* stream);

/* Loss log ring: ring[*counter % capacity] = scale * sum(values[0..n)); ++*counter (one device
 * thread). This is the device-side replacement of mlflow.log_metric("loss", loss.item(), step)
 * (src/server_part.py:55): the slot comes from device memory, so a captured HIP graph logs every
 * replay into a new slot, and the host flushes the ring every N steps instead of syncing per step. */
int slk_loss_log(const float* values, int n, float scale, float* ring, int capacity, int* counter,
                 void* stream);

/* Every optimizer step of one split step in ONE launch: for each segment s < nseg (<= 4),
 * slk_sgd_from_slabs(params[s], grads ? grads[s] : NULL, slabs[s], nslab[s], n[s], lr), and, when
 * loss_values != NULL, slk_loss_log(loss_values, loss_n, loss_scale, ring, capacity, counter) —
 * bit-identical to those separate launches. Replaces the server's optimizer.step() + log_metric
 * (src/server_part.py:52,55) and the client's optimizer.step() (src/client_part.py:133) at the end
 * of a fused split step. The pointer/size arrays are host memory. A segment with params[s] == NULL
 * (and grads[s] != NULL) only reduces: grads[s] = sum of its slabs (the data-parallel replica fills
 * its all-reduce bucket this way: several slk_reduce_slabs in one launch). */
int slk_sgd_multi_from_slabs(float* const* params, float* const* grads, const float* const* slabs,
                             const int* nslab, const int* n, int nseg, float lr, const float* loss_values,
                             int loss_n, float loss_scale, float* ring, int capacity, int* counter,
                             void* stream);

/* MNIST batch from the HBM-resident u8 dataset (replaces DataLoader(batch_size=64, shuffle=True)
 * over torchvision MNIST + ToTensor + Normalize((0.1307,),(0.3081,)), src/client_part.py:61-64,98):
 * x[s] = ((float)images[idx[s]] / 255 - mean) / std as f32 [B,1,28,28], y[s] = labels[idx[s]] (i64).
 * images: [n_images][784] u8 (4-byte aligned); x 16-byte aligned. An idx outside [0, n_images)
 * sets *err_flag (if non-null) and reads image 0. Bit-identical to the torchvision transform. */
int slk_mnist_batch(const uint8_t* images, const uint8_t* labels, int n_images, const int64_t* idx,
                    int B, float mean, float std, float* x, int64_t* y, int* err_flag, void* stream);


/* ================================================================ lossless cut-exchange codec (K3 / K4)
 * The multi-GPU topologies move the cut over RCCL instead of the reference's pickled HTTP body
 * (src/client_part.py:117-125 activations out, src/server_part.py:57-58 gradient back). The cut is a
 * ReLU output (about half zeros), so a micro-batch of n elements travels as mask (ceil(n/32) uint32
 * words: bit set where the element's bit pattern is nonzero) + the set elements in order, and the cut
 * gradient as its values at the same set positions only (the client applies its own ReLU mask, a subset
 * of the set bits, before using the gradient; the left-out positions never reach a result). Blocks of
 * 2048 elements: counts/offsets hold slk_cut_blocks(n) ints, total one int (the number of set bits).
 *   encode : mask, per-block counts, exclusive offsets, total, and the packed values of x;
 *   offsets: counts, offsets, total from a received mask;
 *   pack   : the values of x at the mask's set positions (the gradient direction);
 *   unpack : x = the values scattered to the set positions, zeros elsewhere. */
int slk_cut_blocks(int64_t n);
int slk_cut_encode(const float* x, int64_t n, uint32_t* mask, int* counts, int* offsets, int* total, float* vals,
                   void* stream);
int slk_cut_offsets(const uint32_t* mask, int64_t n, int* counts, int* offsets, int* total, void* stream);
int slk_cut_pack(const float* x, int64_t n, const uint32_t* mask, const int* offsets, float* vals, void* stream);
int slk_cut_unpack(const float* vals, int64_t n, const uint32_t* mask, const int* offsets, float* x, void* stream);
/* Fused consumers of a received micro-batch (the K3 / K4 server; each replaces an unpack or a pack pass over
 * the dense f32 cut, src/server_part.py:39-45 and :57-58):
 *   ranks      : ranks[w] (ceil(n/32) ints) = the vals index of mask word w's first set element
 *                (offsets of the block + the set bits of its earlier words), from slk_cut_offsets' offsets;
 *   unpack_x3  : the x3 input images of B samples (slk_conv2_act16_bytes(B) bytes, each sample at the scale
 *                of act_amax[b]) straight from mask + vals + ranks: the images slk_conv1_fwd_x3 would have
 *                written from the same cut (bit for bit), no dense f32 cut;
 *   dgrad_pack : slk_conv2_dgrad_x3 writing the cut gradient packed (values at the mask's set positions, at
 *                their ranks) — what slk_cut_pack would extract from its dense output. */
int slk_cut_ranks(const uint32_t* mask, int64_t n, const int* offsets, int* ranks, void* stream);
int slk_cut_unpack_x3(const float* vals, const uint32_t* mask, const int* ranks, const float* act_amax, int B,
                      uint16_t* act16, void* stream);
int slk_conv2_dgrad_x3_pack(const float* dpooled, const float* dp_amax, const uint8_t* code, const float* W2,
                            const uint32_t* mask, const int* ranks, float* vals, int B, void* stream);
/* The same over the np parts of one server chunk (one part per client, each n elements / part_b samples) in
 * one launch per pass: `parts` is a device table of pointers (uint64 each) —
 *   offsets_ranks_parts: [np][5] = (mask, counts, offsets, total, ranks): count + scan + ranks of every part;
 *   unpack_x3_parts    : [B / part_b][3] = (vals, mask, ranks); sample b reads part b / part_b;
 *   dgrad_x3_pack_parts: [B / part_b][3] = (mask, ranks, vals). */
int slk_cut_offsets_ranks_parts(const uint64_t* parts, int np, int64_t n, void* stream);
int slk_cut_unpack_x3_parts(const uint64_t* parts, int part_b, const float* act_amax, int B, uint16_t* act16,
                            void* stream);
int slk_conv2_dgrad_x3_pack_parts(const float* dpooled, const float* dp_amax, const uint8_t* code, const float* W2,
                                  const uint64_t* parts, int part_b, int B, void* stream);

/* ================================================================ widened split CNN (BASELINE config 5)
 * The reference has no such model: these entry points run the north star's
 * widened config — client conv1 3->64 (32x32) + ReLU, conv2 64->128 + ReLU + pool, conv3 128->256 +
 * ReLU + pool (the cut, [B,256,8,8]); server Dropout(0.25) + Linear(16384,10) + cross-entropy; Adam —
 * behind the same step contract (client_part.py:110-138 <-> server_part.py:25-58). Oracle:
 * oracle/wide_step.py. Activations are bf16 in the "C8" layout [B][C/8][H][W][8] (8 channels of one
 * pixel = one 16-byte chunk); routing codes are u8 in the same layout (0..3 = argmax position in the
 * 2x2 window, first max wins; 4 = ReLU-blocked). Weight masters are f32 in torch layout; the MFMA
 * convolutions read bf16 shadows built by slk_wide_shadows:
 *   w2f [tap][ci/8][co][8] (128x64)   w2d [8-tap][co/8][ci][8]
 *   w3f [co/128][tap][ci/8][co%128][8] (256x128)   w3d [8-tap][co/8][ci][8]
 * Client flat block: [W1 1728 | b1 64 | W2 73728 | b2 128 | W3 294912 | b3 256]; server: [Wf | bf]. */
#define SLK_WIDE_CLIENT_NPARAM 370816
#define SLK_WIDE_SERVER_NPARAM 163850

/* a1 = bf16(relu(conv1(bf16(x)) + b1)), x f32 NCHW [B,3,32,32]; one bf16 MFMA K-step (K = 27 -> 32);
 * w1b [64][32] bf16 from slk_wide_shadows. a1bits (may be NULL): the ReLU word of every pixel, [B][1024]
 * u64, bit c = (a1[c] > 0) — what slk_wide_conv2_dgrad masks with (8 KB a sample instead of a1's 128 KB). */
int slk_wide_conv1_fwd(const float* x, const uint16_t* w1b, const float* b1, uint16_t* a1, uint64_t* a1bits, int B,
                       void* stream);
/* The same ReLU words from a stored a1 (callers that hold a1 but not its words). */
int slk_wide_relu_bits(const uint16_t* a1, uint64_t* a1bits, int B, void* stream);
/* p2, code2 = pool(relu(conv2(a1) + b2)) — bf16 MFMA implicit GEMM, f32 accumulation. */
int slk_wide_conv2_fwd(const uint16_t* a1, const uint16_t* w2f, const float* b2, uint16_t* p2, uint8_t* code2,
                       int B, void* stream);
/* cut, code3 = pool(relu(conv3(p2) + b3)). The cut is what the client sends (client_part.py:117-125). */
int slk_wide_conv3_fwd(const uint16_t* p2, const uint16_t* w3f, const float* b3, uint16_t* cut, uint8_t* code3,
                       int B, void* stream);
/* Server: dropout (hash of seed, *step, b0 + sample, feature; keep iff hash >= keep_threshold, kept values
 * scaled by keep_scale), fc forward, cross-entropy forward+backward (dlogits scaled by grad_scale), the
 * cut gradient dcut = keep * keep_scale * dlogits @ Wf (bf16, C8) and the fc weight-gradient slabs
 * [slk_wide_head_nslab(B)][163850] = [dWf (torch layout) | dbf]. wf8 = slk_wide_fc_shadow(Wf);
 * work = slk_wide_head_work(B) floats of scratch (the step's dropout bits); b0 = global index of sample 0 (micro-batches and
 * SplitFed slices of one step draw the dropout mask of the concatenated batch). Replaces
 * server_part.py:48-51 + the cut-gradient return (:57) for the widened model. */
int slk_wide_head(const uint16_t* cut, const float* wf8, const float* bf, const int64_t* labels, const int* step,
                  unsigned seed, unsigned keep_threshold, float keep_scale, float grad_scale, float* logits,
                  float* loss_i, float* dlogits, uint16_t* dcut, float* slabs, float* work, int* err_flag, int b0,
                  int B, void* stream);
int slk_wide_head_nslab(int B);
int slk_wide_head_work(int B);
/* slk_wide_head split at the loss, for the module path (WideModelPartB.forward -> criterion ->
 * loss.backward(), server_part.py:48-51): _fwd writes the logits (dropout + fc, the same kernel and
 * sum order as slk_wide_head, so bit-identical logits); _bwd takes dlogits from any loss and writes dcut and the fc slabs
 * exactly as slk_wide_head's last stage. */
int slk_wide_head_fwd(const uint16_t* cut, const float* wf8, const float* bf, const int* step, unsigned seed,
                      unsigned keep_threshold, float keep_scale, float* logits, int b0, int B, void* stream);
int slk_wide_head_bwd(const uint16_t* cut, const float* wf8, const float* dlogits, const int* step, unsigned seed,
                      unsigned keep_threshold, float keep_scale, uint16_t* dcut, float* slabs, int b0, int B,
                      void* stream);
/* Client backward (activations.backward(grads), client_part.py:132), with no unpooled gradient ever
 * stored: conv3's wgrad and dgrad apply conv3's max-pool backward (code3) to the POOLED cut gradient
 * dcut while staging it; conv3 wgrad slabs [nslab][294912 + 256]; dp2 = conv3 dgrad = the gradient of
 * p2 at its own 16 x 16 resolution (bf16, C8); conv2's dgrad and wgrad apply conv2's max-pool backward
 * (code2) to dp2 the same way; conv2 wgrad slabs [nslab][73728 + 128]; da1m = conv2 dgrad masked by
 * a1 > 0 (its ReLU words a1bits, slk_wide_conv1_fwd); conv1 wgrad slabs [nslab][1728 + 64] (bf16(x) operand). Slabs are [dW (torch layout) | db],
 * reduced in fixed order. */
int slk_wide_conv3_wgrad(const uint16_t* dcut, const uint8_t* code3, const uint16_t* p2, float* slabs, int B,
                         void* stream);
int slk_wide_conv3_wgrad_nslab(int B);
int slk_wide_conv3_dgrad(const uint16_t* dcut, const uint8_t* code3, const uint16_t* w3d, uint16_t* dp2, int B,
                         void* stream);
int slk_wide_conv2_wgrad(const uint16_t* dp2, const uint8_t* code2, const uint16_t* a1, float* slabs, int B,
                         void* stream);
int slk_wide_conv2_wgrad_nslab(int B);
/* 1 when the K5 weight gradients run on the 2:4-sparse bf16 MFMA (the max-pool-routed dC), 0 dense. */
int slk_wide_wgrad_form(void);
int slk_wide_conv2_dgrad(const uint16_t* dp2, const uint8_t* code2, const uint16_t* w2d, const uint64_t* a1bits,
                         uint16_t* da1m, int B, void* stream);
int slk_wide_conv1_wgrad(const float* x, const uint16_t* da1m, float* slabs, int B, void* stream);
int slk_wide_conv1_wgrad_nslab(int B);

/* Fixed-order slab reduction + torch.optim.Adam step (amsgrad off, no weight decay) on n floats:
 * t = *step + 1; grad (if non-null) receives the reduced gradient. Replaces optimizer.step() for the
 * widened config (the north star's "fused SGD/Adam"). */
int slk_adam_from_slabs(float* param, float* grad, float* m, float* v, const float* slabs, int nslab, int n,
                        float lr, float beta1, float beta2, float eps, const int* step, void* stream);

/* slk_adam_from_slabs over nseg (<= 4) parameter segments, each with its own slab set, in ONE launch
 * (bit-identical to the separate launches); grads may be NULL or hold NULL entries. The pointer and
 * size arrays are host memory. Replaces the per-parameter loop of the client's optimizer.step()
 * (torch.optim.Adam) for the widened model (src/client_part.py:133's call site). */
int slk_adam_multi_from_slabs(float* const* params, float* const* grads, float* const* m, float* const* v,
                              const float* const* slabs, const int* nslab, const int* n, int nseg, float lr,
                              float beta1, float beta2, float eps, const int* step, void* stream);
/* Rebuild the bf16 weight shadows from the f32 masters: w1b [64][32] (W1 rows, k >= 27 zero) and the
 * MFMA layouts of W2 [128,64,3,3] and W3 [256,128,3,3]. */
int slk_wide_shadows(const float* W1, const float* W2, const float* W3, uint16_t* w1b, uint16_t* w2f, uint16_t* w2d,
                     uint16_t* w3f, uint16_t* w3d, void* stream);
/* wf8[j][(plane*64+pix)*8+k] = Wf[j][(plane*8+k)*64+pix]: the fc weight in the cut's C8 order. */
int slk_wide_fc_shadow(const float* wf, float* wf8, void* stream);
/* ++*counter on the device (the per-stage step counter a captured HIP graph advances). */
int slk_tick(int* counter, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SLK_H */
