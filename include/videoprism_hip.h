/*
 * videoprism_hip.h — C-ABI of the MI355X (gfx950) VideoPrism video-encoder library
 * (libvideoprism_hip.so).
 *
 * The reference (tmoroney/videoprism-mlx) has no native FFI: its drop-in surface is the
 * Python API `models.get_model(name, fprop_dtype=...)` + `model.apply(variables, inputs,
 * train=False, return_intermediate=..., frame_paddings=...)` (videoprism/models.py:268-303,
 * videoprism/encoders.py:411-580) and `models_mlx.load_video_encoder(name, weights_path)`
 * (videoprism/models_mlx.py:146-210).  This header is the boundary those Python entry
 * points (videoprism-mlx_amd/videoprism/) bind through ctypes; any other host language
 * binds the same symbols.
 *
 * Conventions
 *  - Every function returns an int status (VP_OK == 0).  On failure a thread-local
 *    message is available from vp_last_error().  VP_EINVAL carries the same messages the
 *    reference raises as ValueError/AssertionError (e.g. encoders.py:86-90).
 *  - Plain pointers and sizes only.  Device pointers are HIP device memory of the handle's
 *    device; `stream` is a hipStream_t passed as void* (NULL = default stream).
 *  - Parameters are passed once, as HOST fp32 arrays in the reference's own Flax layout
 *    and names (scanned layers, leading L axis), and are repacked by the library into
 *    kernel-ready device buffers owned by the handle.
 *  - vp_forward never allocates, never synchronises: all activations live in the caller's
 *    workspace (size from vp_workspace_bytes); the call is asynchronous on `stream` and
 *    can be captured into a hipGraph.
 *  - A handle is bound to one device and is not thread-safe: calls on one handle must not overlap
 *    (in particular vp_prepare_geometry / vp_prepare_frames, which add to the handle's cached tables,
 *    must not run while vp_forward runs on the same handle).  Different handles -- on one device or
 *    several -- may be driven from different host threads at once: the library's launch state (kernel
 *    attributes, CU counts) is kept per device and set under a lock.
 */
#ifndef VIDEOPRISM_HIP_H_
#define VIDEOPRISM_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VP_ABI_VERSION 5

typedef struct vp_handle vp_handle;

enum vp_status {
  VP_OK = 0,
  VP_EINVAL = 1,   /* bad argument / shape (reference ValueError / assert) */
  VP_ENOMEM = 2,   /* device allocation failed */
  VP_EHIP = 3,     /* HIP runtime error */
  VP_ESTATE = 4,   /* handle not finalized / parameter missing */
  VP_ENOTSUP = 5,  /* valid for the reference but outside this library's kernels */
  VP_ECOMM = 6,    /* RCCL error (vp_comm_*, vp_allgather) */
};

/* VP_U8: video frames as uint8 [0, 255], normalised in the patchify kernel exactly as
 * video_utils.py:94 (float32(v) / 255.0) -- a quarter of the fp32 input bytes. */
enum vp_dtype { VP_F32 = 0, VP_BF16 = 1, VP_U8 = 2 };

/* FactorizedEncoder hyper-parameters: models.py:83-104 CONFIGS / encoders.py:399-408. */
typedef struct vp_config {
  int32_t patch_size;          /* 18 */
  int32_t pos_emb_t;           /* pos_emb_shape[0]: 16 (Base) / 8 (Large) */
  int32_t pos_emb_h;           /* pos_emb_shape[1]: 16 */
  int32_t pos_emb_w;           /* pos_emb_shape[2]: 16 */
  int32_t model_dim;           /* 768 / 1024 */
  int32_t num_spatial_layers;  /* 12 / 24 */
  int32_t num_temporal_layers; /* 4 */
  int32_t num_heads;           /* 12 / 16 (dim_per_head must be 64) */
  int32_t mlp_dim;             /* 3072 / 4096 */
  float atten_logit_cap;       /* 50.0 */
  int32_t fprop_dtype;         /* VP_F32 (reference default) or VP_BF16 (get_model(fprop_dtype=bf16)) */
} vp_config;

/* Last error message of the calling thread ("" if none). */
const char* vp_last_error(void);
int vp_abi_version(void);

/* Replaces models.get_model(...) (models.py:268-303): binds a config to a device. */
int vp_create(const vp_config* cfg, int device, vp_handle** out);
int vp_destroy(vp_handle* h);

/* One parameter leaf, by its Flax path under 'params' ('/'-joined, utils.py:84-105), e.g.
 *   "patch_projection/linear/kernel"                                    [P*P*3, D]
 *   "spatial_encoder/transformers_stack/x_layers/self_attention/query/w" [L, D, N, H]
 * host_data: fp32, C-contiguous.  Shapes are validated against the config. */
int vp_set_param(vp_handle* h, const char* name, const float* host_data, const int64_t* shape,
                 int ndim);
/* Number of leaves the config expects (40 for a scanned FactorizedEncoder,
 * encoders_test.py:170) and the i-th leaf's name. */
int vp_param_count(const vp_handle* h, int* count);
int vp_param_name(const vp_handle* h, int index, const char** name);
/* Validates that every leaf was set and uploads the packed weights (one-off). */
int vp_finalize(vp_handle* h);

/* Frames whose patch grid (H/P, W/P) differs from pos_emb_shape[1:]: interpolates the spatial
 * positional table the way encoders.py:497-512 does (_interpolate_emb_2d, jax.image.resize
 * 'bilinear', antialiased when shrinking) and caches it on the device (allocates; call once per
 * new frame size before vp_forward, which never allocates). */
int vp_prepare_geometry(vp_handle* h, int64_t H, int64_t W);

/* Clips of T frames: the temporal positional table resampled to T the way encoders.py:543-553
 * does (_interpolate_emb_1d, :107-130, jax.image.resize 'bilinear', antialiased when shrinking).
 * vp_finalize precomputes T = 1..32; any other T needs one call before vp_forward (allocates one
 * [T][D] fp32 table per distinct T, kept until vp_destroy; idempotent).  1 <= T <= 2^20. */
int vp_prepare_frames(vp_handle* h, int64_t T);

/* Workspace needed by vp_forward for inputs [B, T, H, W, 3]. */
int vp_workspace_bytes(const vp_handle* h, int64_t B, int64_t T, int64_t H, int64_t W,
                       size_t* bytes);

/* Replaces FactorizedEncoder.__call__ (encoders.py:411-456) / model.apply(..., train=False).
 *   video          device [B, T, H, W, 3], in_dtype VP_F32 or VP_BF16 (values as given) or VP_U8
 *   frame_paddings device [B, T] fp32 (1 = padded frame) or NULL (encoders.py:440-447)
 *   out            device [B, T*N, D] embeddings in out_dtype (token = t*N + n, :570-572)
 *   spatial_out    device [B, T*N, D] 'spatial_features' in out_dtype, or NULL (:574-578)
 */
int vp_forward(vp_handle* h, const void* video, int in_dtype, int64_t B, int64_t T, int64_t H,
               int64_t W, const float* frame_paddings, void* out, int out_dtype,
               void* spatial_out, void* workspace, size_t ws_bytes, void* stream);

/* ---------------- HIP-event profiler (bench.py's live per-kernel timing) ----------------
 * vp_profile_enable(h, n): the next n kernel launches of vp_forward are bracketed by
 * hipEventRecord on the launch stream (0 disables).  vp_profile_read syncs on the last event
 * and returns, per kernel class (vp_profile_class_name), the summed milliseconds, algorithmic
 * FLOPs and bytes and the launch count since the previous read, then resets. */
int vp_profile_enable(vp_handle* h, int capacity);
int vp_profile_read(vp_handle* h, int nclass, double* ms, double* flops, double* bytes,
                    int64_t* launches);
/* Only launches of the classes whose bit is set in class_mask get events (default: all).  Each
 * event pair costs the stream a little, so bench.py times the dominant class alone in its timed
 * region and takes the per-class breakdown from a separate profiled step. */
int vp_profile_set_mask(vp_handle* h, uint32_t class_mask);
int vp_profile_class_count(void);
int vp_profile_class_name(int cls, const char** name);
/* Demangled symbol of the kernel most recently launched for class `cls` on this handle ("" if
 * none yet), e.g. "void vp::(anonymous namespace)::gemm_bf16_w4_kernel<9, 512, 0>(...)": bench.py
 * matches PMC traffic records to exactly this kernel.  Valid until the next call for `cls`. */
int vp_profile_kernel_name(vp_handle* h, int cls, const char** name);

/* ---------------- op-level entry points (kernel parity tests, benches) ---------------- */

/* C[M,N] = A[M,K].W[N,K]^T + bias with epilogue:
 *   0 store (out dtype = precision), 1 GELU(erf) [* (1-rowpad)], 2 out_f32 = resid_f32 + (.)*(1-rowpad),
 *   3 out_f32 = (.) + pos[m % pos_rows], 4 = 2 (separate kernel symbol used for ffn_layer2),
 *   5 / 6 / 7 = 2 / 3 / 4 with a bf16 residual stream (bf16 resid and out; precision VP_BF16 only).
 *   precision VP_BF16: A,W bf16; VP_F32: A,W fp32.
 * Replaces layers.py:273-313 (Dense) and :433-499 (einsum projections). */
int vp_op_gemm(int precision, int epilogue, const void* A, int64_t lda, const void* W, int64_t ldw,
               int64_t M, int64_t N, int64_t K, void* out, int64_t ldo, const float* bias,
               const void* resid, int64_t ldr, const float* pos, int64_t pos_rows,
               const float* rowpad, void* stream);

/* Capped attention over rows qkv[num_seq*S, 3*heads*64] = [q|k|v] (q pre-scaled), writing
 * o[num_seq*S, heads*64].  Replaces DotProductAttention._dot_atten (layers.py:601-661).
 * precision VP_BF16 (S <= 256: the spatial kernel at S == 256, the temporal kernel at S <= 16,
 * the sequence-packed kernel between; any S > 256 without key_pad: the long-sequence kernel of the LvT
 * auxiliary encoder; S > 256 with key_pad: the online-softmax kernel of vp_op_attention_masked, as the
 * forward runs it) or VP_F32 (S <= 256).  key_pad: [num_seq*S] or NULL.
 * bf16 with a cap outside (0, 50] (no capping, or one whose unnormalised fp32 numerators could
 * overflow) runs the online-softmax kernel of vp_op_attention_masked, any S. */
int vp_op_attention(int precision, const void* qkv, void* o, int64_t num_seq, int64_t S,
                    int64_t heads, float cap, const float* key_pad, void* stream);

/* LayerNorm (layers.py:208-270) of fp32 or bf16 rows (in_dtype) with gamma = 1 + scale; optional
 * row permutation (0 none, 1 (b t n)->(b n t), 2 (b n t)->(b t n)) and fp32 add[t][D] by output t. */
int vp_op_layernorm(const void* x, int in_dtype, int64_t rows, int64_t D, const float* gamma,
                    const float* beta, void* out, int out_dtype, int perm, int64_t T, int64_t Nsp,
                    const float* add, void* stream);

/* _image_to_patch (encoders.py:70-104): video [BT,H,W,C] -> patches [BT*(H/P)*(W/P), kpad]
 * with features in (p, q, c) order and zero padding from P*P*C to kpad. */
int vp_op_patchify(const void* video, int in_dtype, void* patches, int out_dtype, int64_t BT,
                   int64_t H, int64_t W, int64_t C, int64_t P, int64_t kpad, void* stream);

/* Build-defined pooled clip embedding used by the multi-GPU gather (the video-only encoder
 * has no pooler in the reference): out[b] = l2norm(mean_l emb[b, l, :]) in fp32, with the
 * reference's _l2_normalize (encoders.py:50-67, eps 1e-12). */
int vp_op_pool_l2(const void* emb, int dtype, int64_t B, int64_t L, int64_t D, float* out,
                  void* stream);

/* Attention over rows qkv[num_seq*S, 3*heads*64] (q pre-scaled), any S, with key paddings
 * key_pad [num_seq*S] (nullable) and, if causal, the merged causal + padding mask of
 * layers.py:111-179 (a padded query row is fully masked -> uniform weights).  qkv / o in
 * `precision` (VP_F32 or VP_BF16).  cap <= 0 disables the tanh cap.  Used by the text tower: bf16
 * with 16 < S <= 256 and 0 < cap <= 50 on the sequence-packed MFMA kernel, otherwise fp32 math with an
 * online softmax. */
int vp_op_attention_masked(int precision, const void* qkv, void* o, int64_t num_seq, int64_t S,
                           int64_t heads, float cap, const float* key_pad, int causal, void* stream);

/* video_emb [B, D] . text_emb [Q, D]^T -> out [B, Q] (fp32): the video-text similarity of the
 * LvT models (README / colab usage of FactorizedVideoCLIP's embeddings). */
int vp_op_similarity(const float* video_emb, const float* text_emb, int64_t B, int64_t Q, int64_t D,
                     float* out, void* stream);

/* ---------------- LvT video-text model: FactorizedVideoCLIP (encoders.py:762-910) ----------------
 * Replaces models.get_model('videoprism_lvt_public_v1_{base,large}') + model.apply(variables,
 * inputs, text_token_ids, text_paddings, train=False, normalize, return_intermediate,
 * frame_paddings) (models.py:116-212, 268-303).  Parameters are the Flax leaves under 'params':
 * 'vision_encoder/...' (the FactorizedEncoder leaves above), 'auxiliary_encoder/...',
 * 'contrastive_vision_pooler/...', 'text_encoder/...' (88 leaves for a scanned model,
 * encoders_test.py:339).  Same conventions as vp_handle (borrowed device pointers, async on
 * `stream`, no allocation in the encode calls, one device per handle, not thread-safe). */
typedef struct vp_clip vp_clip;

typedef struct vp_clip_config {
  vp_config video;               /* vision encoder hyper-parameters (models.py:116-145) */
  int32_t num_auxiliary_layers;  /* 2: VisionTransformer over all T*N tokens (:846-857) */
  int32_t vocabulary_size;       /* 32000 (c4_en, models.py:55-60) */
  int32_t num_unimodal_layers;   /* 12: text tower depth */
  int32_t enable_causal_atten;   /* 1 */
} vp_clip_config;

int vp_clip_create(const vp_clip_config* cfg, int device, vp_clip** out);
int vp_clip_destroy(vp_clip* c);
int vp_clip_set_param(vp_clip* c, const char* name, const float* host_data, const int64_t* shape,
                      int ndim);
int vp_clip_param_count(const vp_clip* c, int* count);
int vp_clip_param_name(const vp_clip* c, int index, const char** name);
int vp_clip_finalize(vp_clip* c);
/* The vision tower's vp_handle (owned by the clip): vp_profile_* on it also covers the
 * auxiliary encoder and pooler launches of vp_clip_encode_video. */
int vp_clip_video_handle(vp_clip* c, vp_handle** video);

/* Video side of FactorizedVideoCLIP.__call__ (encoders.py:833-885):
 *   video_emb      device [B, D] fp32: contrastive_vision_pooler(auxiliary_encoder(features)),
 *                  L2-normalised if `normalize` (:859-872)
 *   frame_emb      device [B, T, D] fp32 'frame_embeddings' (pooler per frame, :874-885) or NULL
 *   spatial_out    device [B, T*N, D] 'spatial_features' in out_dtype, or NULL
 *   spatiotemporal_out device [B, T*N, D] 'spatiotemporal_features' (the vision encoder's output,
 *                  :844-845) in the handle's fprop dtype (out_dtype must match), or NULL */
int vp_clip_video_workspace_bytes(const vp_clip* c, int64_t B, int64_t T, int64_t H, int64_t W,
                                  size_t* bytes);
int vp_clip_encode_video(vp_clip* c, const void* video, int in_dtype, int64_t B, int64_t T,
                         int64_t H, int64_t W, const float* frame_paddings, int normalize,
                         float* video_emb, float* frame_emb, void* spatial_out,
                         void* spatiotemporal_out, int out_dtype, void* workspace,
                         size_t ws_bytes, void* stream);

/* Text side (encoders.py:887-908): ids device int32 [Q, L], paddings device fp32 [Q, L]
 * (1 = padded token); text_emb device [Q, D] fp32 = the CLS token after unimodal_ln,
 * L2-normalised if `normalize`.  Out-of-range ids are clamped (JAX gather semantics). */
int vp_clip_text_workspace_bytes(const vp_clip* c, int64_t Q, int64_t L, size_t* bytes);
int vp_clip_encode_text(vp_clip* c, const int32_t* ids, const float* paddings, int64_t Q,
                        int64_t L, int normalize, float* text_emb, void* workspace,
                        size_t ws_bytes, void* stream);

/* ---------------- video classifier: FactorizedVideoClassifier (encoders.py:583-653) ----------------
 * Replaces encoders.FactorizedVideoClassifier(encoder_params, num_classes).apply(...) and the
 * models.videoprism_vc_v1_{base,large}(num_classes) builders (models.py:195-216).  Leaves:
 * 'encoder/...' (the FactorizedEncoder leaves), 'atten_pooler/...' (AttenTokenPoolingLayer with
 * hidden D, 12 leaves), 'projection/linear/{kernel [D, C], bias [C]}': 54 in all
 * (encoders_test.py:224).
 *   logits      device [B, num_classes] fp32
 *   embeddings  device [B, D] fp32 'global_embeddings' (the pooled vector) or NULL
 *   spatial_out / spatiotemporal_out as vp_clip_encode_video */
typedef struct vp_classifier vp_classifier;
int vp_classifier_create(const vp_config* cfg, int num_classes, int device, vp_classifier** out);
int vp_classifier_destroy(vp_classifier* c);
int vp_classifier_set_param(vp_classifier* c, const char* name, const float* host_data,
                            const int64_t* shape, int ndim);
int vp_classifier_param_count(const vp_classifier* c, int* count);
int vp_classifier_param_name(const vp_classifier* c, int index, const char** name);
int vp_classifier_finalize(vp_classifier* c);
int vp_classifier_video_handle(vp_classifier* c, vp_handle** video);
int vp_classifier_workspace_bytes(const vp_classifier* c, int64_t B, int64_t T, int64_t H, int64_t W,
                                  size_t* bytes);
int vp_classifier_forward(vp_classifier* c, const void* video, int in_dtype, int64_t B, int64_t T,
                          int64_t H, int64_t W, const float* frame_paddings, float* logits,
                          float* embeddings, void* spatial_out, void* spatiotemporal_out,
                          int out_dtype, void* workspace, size_t ws_bytes, void* stream);

/* ---------------- multi-GPU: RCCL all-gather of pooled clip embeddings ----------------
 * The reference runs on one device; its video-text usage scores every clip against every query,
 * `similarities = video_emb @ text_emb.T` (README.md:81, verify_clip_models.py:84).  With clips
 * sharded by batch over one process per GPU, that step needs every rank's
 * [b, D] video embeddings on every rank: one all-gather over xGMI.  The communicator is RCCL's:
 * rank 0 creates a unique id (vp_comm_unique_id, vp_comm_id_bytes() bytes), the host sends it to
 * every rank by any channel (videoprism/distributed.py uses torch.distributed), and every rank
 * calls vp_comm_init with it (collective: blocks until all nranks joined).
 * vp_allgather: recv[r*count .. (r+1)*count) = rank r's send[0 .. count) on every rank, dtype
 * VP_F32 / VP_BF16 / VP_U8, asynchronous on `stream` (device pointers of the comm's device).
 * `count` must be the same on every rank (RCCL's contract): hosts with uneven shards pad to the
 * largest (videoprism/distributed.py Communicator.all_gather_rows).  Every vp_comm_* entry point
 * leaves the calling thread's current HIP device as it found it. */
typedef struct vp_comm vp_comm;
int vp_comm_id_bytes(void);
int vp_comm_unique_id(uint8_t* id_out, int64_t nbytes);
int vp_comm_init(const uint8_t* id, int64_t nbytes, int nranks, int rank, int device, vp_comm** out);
int vp_comm_destroy(vp_comm* c);
int vp_allgather(vp_comm* c, const void* send, void* recv, int64_t count, int dtype, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* VIDEOPRISM_HIP_H_ */
