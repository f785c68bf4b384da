/*
 * spk_hip.h — C ABI of libspk_hip.so, the MI355X (gfx950) speaker-embedding hot path.
 *
 * Plain C, POD arguments only: device pointers are raw `float*`/`int64_t*` (owned by the
 * caller, e.g. the torch caching allocator), streams are `hipStream_t` passed as `void*`.
 * Every entry point returns 0 on success or a negative SPK_E_* code; the message of the
 * last failure on the calling thread is available from spk_last_error().  No C++
 * exception crosses this boundary.  Handles are immutable after creation, so one handle
 * may be used from several streams concurrently, each forward with its own workspace (all
 * per-forward state, the fp16x3 range word included, lives in the workspace); forward()
 * allocates nothing (the caller provides a workspace sized by spk_model_workspace_bytes())
 * and never synchronises the host, so it can be captured into a hipGraph.
 *
 * Which reference interface each entry point replaces (paths relative to the reference
 * repo nanless/3D-Speaker):
 *   spk_fbank_f32        speakerlab/process/processor.py:133-158 (FBank.__call__ ->
 *                        torchaudio.compliance.kaldi.fbank) and the C++ runtime's
 *                        FbankComputer::compute_feature runtime/onnxruntime/feature/feature_fbank.cpp:22-91
 *   spk_model_create     model construction + strict load_state_dict in
 *                        speakerlab/bin/infer_sv_batch.py:247-253 (and the ONNX session
 *                        runtime/onnxruntime/model/speaker_embedding_model.cpp:7-40)
 *   spk_model_forward    nn.Module.forward of ERes2NetV2.py:235-254, ERes2Net.py:208-231,
 *                        ECAPA_TDNN.py:430-463, DTDNN.py:111-115 (and
 *                        OnnxSpeakerEmbeddingModel::extract_embedding speaker_embedding_model.cpp:42-69)
 *   spk_cosine_affinity  sklearn cosine_similarity as used by speakerlab/process/cluster.py:59-62,150
 *                        and speakerlab/bin/compute_score_metrics.py:110-114
 *   spk_cosine_topk      the consumers of the row-block affinity: best matches
 *                        per row / threshold counts, the affinity never materialised
 *   spk_cosine_trials    the per-trial cosine_similarity loop of compute_score_metrics.py:102-118
 */
#ifndef SPK_HIP_H
#define SPK_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPK_OK 0
#define SPK_E_INVALID (-1)     /* bad argument / shape */
#define SPK_E_HIP (-2)         /* HIP runtime error */
#define SPK_E_WEIGHTS (-3)     /* missing or mis-shaped state_dict tensor */
#define SPK_E_DEVICE (-4)      /* handle used on another device */
#define SPK_E_WORKSPACE (-5)   /* workspace too small */
#define SPK_E_UNSUPPORTED (-6)

/* architectures (the four models on the north-star path) */
#define SPK_ARCH_ERES2NETV2 1  /* speakerlab.models.eres2net.ERes2NetV2.ERes2NetV2 */
#define SPK_ARCH_ERES2NET 2    /* speakerlab.models.eres2net.ERes2Net.ERes2Net     */
#define SPK_ARCH_ECAPA 3       /* speakerlab.models.ecapa_tdnn.ECAPA_TDNN.ECAPA_TDNN */
#define SPK_ARCH_CAMPPLUS 4    /* speakerlab.models.campplus.DTDNN.CAMPPlus         */
#define SPK_ARCH_RESNET 5      /* speakerlab.models.resnet.ResNet.ResNet (BasicBlock, TSTP) */
#define SPK_ARCH_RES2NET 6     /* speakerlab.models.res2net.Res2Net.Res2Net (TSTP)  */

typedef struct spk_model spk_model_t;

/* One state_dict tensor, HOST memory, float32 contiguous (int tensors such as
 * num_batches_tracked may be passed with data == NULL).  Keys are the reference's. */
typedef struct {
  const char* name;
  const float* data;
  int32_t ndim;
  int64_t shape[4];
} spk_weight_t;

/* Constructor arguments of the reference module (only those that shape the graph). */
#define SPK_PRECISION_FP32 0
#define SPK_PRECISION_FP16 1
#define SPK_POOL_TSTP 0
#define SPK_POOL_TAP 1
#define SPK_POOL_TSDP 2
#define SPK_POOL_ASTP 3

typedef struct {
  int32_t arch;
  int32_t feat_dim;       /* 80 */
  int32_t embed_dim;      /* embedding_size / lin_neurons */
  int32_t m_channels;     /* ERes2Net*: m_channels */
  int32_t base_width;     /* ERes2NetV2: baseWidth (26); ERes2Net: 32 */
  int32_t scale;          /* ERes2Net*: scale (2) */
  int32_t expansion;      /* ERes2Net*: expansion (2) */
  int32_t two_emb_layer;  /* ERes2Net*: two_emb_layer */
  int32_t channels[5];    /* ECAPA: channels */
  int32_t kernel_sizes[5];/* ECAPA: kernel_sizes */
  int32_t dilations[5];   /* ECAPA: dilations */
  int32_t precision;      /* SPK_PRECISION_FP32 (0, default): fp32-accurate (fp16x3 split
                             products); SPK_PRECISION_FP16 (1): one fp16 MFMA product per
                             multiply, fp32 accumulation -- BASELINE config C3's reduced-
                             precision mode (cosine >= 0.9999 to the reference) */
  int32_t pooling;        /* ERes2Net*: pooling_func -- SPK_POOL_TSTP (0, default), SPK_POOL_TAP (1),
                             SPK_POOL_TSDP (2), SPK_POOL_ASTP (3, global_context_att=False)
                             (pooling_layers.py:10-104) */
  int32_t reserved[6];
} spk_model_config_t;

/* ABI revision: 2 (spk_model_range_check's seven-argument form, spk_model_config_t.pooling) */
int spk_version(void);
const char* spk_last_error(void);

/* Kaldi log-mel Fbank of a ragged batch.  wav: device float32 samples of all utterances
 * back to back; wav_offsets/frame_offsets: DEVICE int64 arrays of n_utt+1 entries (sample
 * and frame starts; frames = 1 + (len-400)/160).  feats: device [total_frames, n_mels]. */
int spk_fbank_f32(const float* wav, const int64_t* wav_offsets, int32_t n_utt, float* feats,
                  const int64_t* frame_offsets, int32_t n_mels, int32_t mean_nor, void* stream);

/* Same, written as a zero-padded batch [n_utt, t_max, n_mels]: utterance u at rows
 * [u * t_max, u * t_max + frames_u) (frames_u from frame_offsets), its remaining rows 0.
 * The input of spk_model_forward_lengths for variable-length batches. */
int spk_fbank_f32_padded(const float* wav, const int64_t* wav_offsets, int32_t n_utt, float* feats,
                         const int64_t* frame_offsets, int32_t t_max, int32_t n_mels, int32_t mean_nor, void* stream);

/* Build a handle on the CURRENT HIP device: folds BatchNorm into conv weights, packs them
 * for the kernels and uploads them (synchronous, once per model). */
int spk_model_create(const spk_model_config_t* cfg, const spk_weight_t* weights, int32_t n_weights,
                     spk_model_t** out);
int spk_model_destroy(spk_model_t* model);

/* Workspace bytes needed by spk_model_forward for a [B, T, feat_dim] batch. */
int spk_model_workspace_bytes(spk_model_t* model, int32_t B, int32_t T, size_t* bytes);

/* feats: device [B, T, feat_dim] float32; emb_out: device [B, embed_dim] float32. */
int spk_model_forward(spk_model_t* model, const float* feats, int32_t B, int32_t T, void* workspace,
                      size_t workspace_bytes, float* emb_out, void* stream);

/* Variable-length batch: feats is [B, T, feat_dim] with utterance b occupying frames
 * [0, lengths[b]) (lengths: DEVICE int32 [B]).  lengths == NULL is spk_model_forward.
 *  - CAM++ (2 <= lengths[b] <= T): frames past lengths[b] are
 *    ignored, every embedding equals the forward of that utterance alone (no padding
 *    enters the computation).  Replaces running DTDNN.py:111-115 once per utterance.
 *  - ECAPA-TDNN (1 <= lengths[b] <= T): the reference's forward(x, lengths)
 *    (ECAPA_TDNN.py:209-287, 430-454): the convolutions run over the padded batch, the SE
 *    squeeze means and the attentive-pooling statistics cover frames [0, lengths[b]) only.
 *    (The reference takes RELATIVE lengths; the Python module converts them with the
 *    reference's own mask arithmetic, length_to_mask :11-27.)
 * Other architectures return SPK_E_UNSUPPORTED for a non-NULL lengths. */
int spk_model_workspace_bytes_lengths(spk_model_t* model, int32_t B, int32_t T, int32_t ragged, size_t* bytes);
int spk_model_forward_lengths(spk_model_t* model, const float* feats, int32_t B, int32_t T, const int32_t* lengths,
                              void* workspace, size_t workspace_bytes, float* emb_out, void* stream);

/* fp16x3 range guard, resolved on the device.  The default kernels represent every GEMM
 * operand as two fp16 values (fp32-accurate, csrc/conv_gemm.hip); a value at or past fp16's
 * range (65504) would saturate.  Every producer of an unbounded activation (and the input
 * check) raises a range word in the caller's workspace -- one per forward, zeroed when the
 * forward starts -- to the largest value it wrote once that reaches 2^14.  ECAPA-TDNN and
 * CAM++ GEMMs then split their operands scaled by a power of two taken from the word (exact,
 * no re-run); ERes2Net* / ResNet re-run the flagged plan segment on exact-fp32 MFMA kernels,
 * launched behind it on the same stream and gated on that word.  spk_model_forward* therefore
 * only enqueue (no host synchronisation), and concurrent forwards on different streams with
 * different workspaces never see each other's word.  spk_model_range_check() reports
 * (synchronising `stream`) whether the word of the last forward of shape (B, T, ragged) that
 * used `workspace` was set (diagnostics).  spk_model_forward_exact() (same arguments as
 * spk_model_forward_lengths, lengths may be NULL) runs the exact plan only.  A handle whose
 * packed weights leave fp16's range always runs exact.  The workspace queries cover both
 * plans. */
int spk_model_range_check(spk_model_t* model, int32_t B, int32_t T, int32_t ragged, const void* workspace,
                          void* stream, int32_t* overflowed);
int spk_model_forward_exact(spk_model_t* model, const float* feats, int32_t B, int32_t T, const int32_t* lengths,
                            void* workspace, size_t workspace_bytes, float* emb_out, void* stream);
/* How the guarded forward of shape (B, T, ragged) is cut (diagnostics, tests): the exact
 * re-run is captured per segment of the plan, right behind the segment it can replace, and
 * only for segments with a split-GEMM operand not statically bounded below 2^14 (ERes2Net*:
 * Hardtanh / weight-norm bounds leave only the stem's segment; ResNet: one segment, the whole
 * plan; ECAPA-TDNN / CAM++: scaled split, one segment, no twin).  n_segments: segments of the
 * plan; n_twin_segments: those with an exact twin; n_gated_steps: launches of the exact plan
 * enqueued behind every guarded forward (no-ops unless the range word is set); 0 / 0 / 0 for
 * an exact-only handle. */
int spk_model_guard_plan(spk_model_t* model, int32_t B, int32_t T, int32_t ragged, int32_t* n_segments,
                         int32_t* n_twin_segments, int32_t* n_gated_steps);

/* Algorithmic FLOPs per utterance of T frames (2 x conv/linear MACs). */
int spk_model_flops(spk_model_t* model, int32_t T, double* flops);

/* Introspection / measurement of the launch plan for a [B, T] batch: number of steps,
 * each step's name, the kernel it launches (rocprofv3 naming) and its algorithmic FLOPs;
 * spk_model_forward_timed() is spk_model_forward() with a HIP event around every step
 * (synchronises; used by bench.py for the roofline figure, not for throughput). */
int spk_model_plan_size(spk_model_t* model, int32_t B, int32_t T, int32_t* n_steps);
int spk_model_plan_step(spk_model_t* model, int32_t B, int32_t T, int32_t i, char* name, int32_t name_len,
                        char* kernel, int32_t kernel_len, double* flops);
/* Algorithmic HBM bytes of plan step i (every operand read / written once, fp32; conv
 * steps only, 0 for steps that are not priced): the byte side of the per-launch roofline. */
int spk_model_plan_step_bytes(spk_model_t* model, int32_t B, int32_t T, int32_t i, double* bytes);
int spk_model_forward_timed(spk_model_t* model, const float* feats, int32_t B, int32_t T, void* workspace,
                            size_t workspace_bytes, float* emb_out, void* stream, float* step_ms,
                            int32_t max_steps);

/* out[i*ldo + j] = <Ea_i, Eb_j> / (max(|Ea_i|,eps) * max(|Eb_j|,eps)), device pointers,
 * row-major [Na,E] and [Nb,E] float32.  Matches sklearn cosine_similarity (normalize with
 * zero-norm rows left as zero). */
int spk_cosine_affinity(const float* Ea, int64_t Na, const float* Eb, int64_t Nb, int32_t E, float* out,
                        int64_t ldo, void* stream);

/* Consumers of the cosine affinity, applied where each tile is produced (the N x Nb matrix is
 * never written): for every row i of Ea, the k best (score, column) pairs over Eb, ordered by
 * score descending then column ascending, and the number of columns with score >= threshold.
 * exclude_self drops column i + self_offset of row i (a rank's row block [r0, r1) of the
 * all-gathered embeddings: self_offset = r0).  Outputs (device, any may be NULL):
 * top_scores [Na][k] float32, top_index [Na][k] int64 (-1 when fewer than k columns),
 * count_ge [Na] int64.  workspace: device, spk_cosine_topk_workspace_bytes(Na, Nb). */
#define SPK_CONSUME_TOPK 1
typedef struct {
  int32_t kind;            /* SPK_CONSUME_TOPK */
  int32_t k;               /* 1..8 */
  int32_t exclude_self;
  int64_t self_offset;
  float threshold;
  float* top_scores;
  int64_t* top_index;
  int64_t* count_ge;
  void* workspace;
  size_t workspace_bytes;
} spk_affinity_consumer_t;
int spk_cosine_topk_workspace_bytes(int64_t Na, int64_t Nb, size_t* bytes);
int spk_cosine_topk(const float* Ea, int64_t Na, const float* Eb, int64_t Nb, int32_t E,
                    const spk_affinity_consumer_t* consumer, void* stream);

/* Trial scoring: scores[t] = cosine(Ea[ia[t]], Eb[ib[t]]) for n_trials (enrol, test) index
 * pairs (device int64 arrays), sklearn semantics (zero-norm rows divide by 1). */
int spk_cosine_trials(const float* Ea, const float* Eb, int32_t E, const int64_t* ia, const int64_t* ib,
                      int64_t n_trials, float* scores, void* stream);

/* Spectral clustering preparation (reference cluster.py SpectralCluster.p_pruning :64-77
 * and get_laplacian :79-84): S is the N x N cosine affinity (row stride lds); every row's
 * n_elems smallest entries are zeroed (ties at the threshold lowest index first), the
 * result symmetrised, its diagonal zeroed, and L = diag(row |sums|) - M written to L (row
 * stride ldl).  workspace: N*N floats (device). */
int spk_spectral_laplacian(const float* S, int64_t N, int64_t lds, int32_t n_elems, float* L, int64_t ldl,
                           void* workspace, size_t workspace_bytes, void* stream);

/* All eigenpairs of a symmetric N x N matrix (rocSOLVER ssyevd; replaces ARPACK eigsh in
 * cluster.py:88-89): eigenvalues ascending into w (device, N), eigenvector k overwrites row
 * k of A (row-major, stride lda).  Synchronises the stream. */
int spk_symmetric_eig(float* A, int64_t N, int64_t lda, float* w, void* stream);


#ifdef __cplusplus
}
#endif

#endif /* SPK_HIP_H */
