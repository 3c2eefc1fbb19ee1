/*
 * libavc — MI355X (gfx950) adversarial-perturbation engine for AdaIN-VC.
 *
 * C ABI: plain pointers and sizes, no torch / HIP C++ types in signatures.
 * This is the boundary behind the reference's Python attack functions:
 *
 *   avc_emb_attack   replaces  attack_utils.emb_attack   (/root/reference/attack_utils.py:51-86)
 *   avc_*_attack_emb the same with adv_tgt embedded beforehand (an adv_tgt of another length:
 *                    attack_utils.py:74-75 / 117-119 embed it on its own, attack.py:49-56 loads
 *                    each input from its own wav)
 *   avc_se_forward   replaces  SpeakerEncoder.forward    (/root/reference/models.py:327-343)
 *   avc_create       replaces  AdaInVC(config) + load_state_dict of the speaker encoder
 *                              (/root/reference/data_utils.py:219-221, models.py:213-283)
 *   avc_e2e_attack   replaces  attack_utils.e2e_attack   (/root/reference/attack_utils.py:7-48)
 *   avc_fb_attack    replaces  attack_utils.fb_attack    (/root/reference/attack_utils.py:89-130)
 *   avc_inference    replaces  AdaInVC.inference         (/root/reference/models.py:472-489)
 *   avc_attach_vc    replaces  load_state_dict of content_encoder / decoder (models.py:121-208, 346-435)
 *   avc_pm_forward   replaces  PredictiveModel.forward   (/root/reference/models/predictive_model.py:87-110)
 *   avc_vsmask_protect replaces VSMask._protect_waveform's mel loop (/root/reference/vsmask.py:177-208)
 *   avc_vsmask_apply_header replaces UniversalPerturbationHeader.apply_header (models/header_model.py:70-95)
 *   avc_header_optimize replaces UniversalPerturbationHeader.optimize (models/header_model.py:25-68)
 *   avc_dsp_wav2mel  replaces  data_utils.file2mel after load/trim (+ normalize) (/root/reference/data_utils.py:65-118, 35-47)
 *   avc_dsp_mel2wav  replaces  data_utils.mel2wav (+ denormalize)   (/root/reference/data_utils.py:121-165, 50-62)
 *   avc_dsp_griffin_lim replaces data_utils.griffin_lim            (/root/reference/data_utils.py:168-197)
 *   avc_dsp_mel_basis   replaces librosa.filters.mel / data_utils.inv_mel_matrix (data_utils.py:16-32, 110)
 *
 * The reference has no native code and no FFI of its own; the Python binding a
 * maintainer would add is shown in INTEGRATION.md (ctypes).
 *
 * Conventions
 *   - every tensor argument is a DEVICE pointer to contiguous fp32 data in the
 *     reference's [B, C, T] layout (torch .contiguous() tensors' data_ptr()),
 *     owned by the caller;  the library owns its workspace (grow-only, per ctx).
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream); all
 *     work is enqueued on it; calls return after enqueueing (asynchronous).
 *   - return 0 on success, non-zero on error; avc_last_error() then returns a
 *     thread-local message.  The Python layer raises RuntimeError(message).
 *   - one ctx per device; distinct ctx are independent and may be driven from
 *     different host threads.  A single ctx is not reentrant.
 */
#ifndef AVC_H
#define AVC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AVC_MAX_BLOCKS 16

/* SpeakerEncoder hyper-parameters, config.yaml model.SpeakerEncoder
 * (/root/reference/models.py:218-232).  act: 0 = ReLU, 1 = LeakyReLU(0.01). */
typedef struct avc_se_cfg {
    int32_t c_in, c_h, c_out, kernel_size;
    int32_t bank_size, bank_scale, c_bank;
    int32_t n_conv_blocks, n_dense_blocks;
    int32_t subsample[AVC_MAX_BLOCKS];
    int32_t act;
} avc_se_cfg;

/* Arithmetic of the per-iteration loop.  FP32: exact-f32 MFMA (v_mfma_f32_16x16x4_f32 in the fused /
 * long engines, avc_fused_core.h); BF16: v_mfma_f32_16x16x32_bf16 operands, fp32 accumulation,
 * fp32 InstanceNorm statistics, loss and Adam state. */
enum { AVC_PREC_FP32 = 0, AVC_PREC_BF16 = 1 };

/* Loss reduction over a batch of B utterances.
 *  INDEPENDENT: each utterance is its own attack (loss summed over utterances,
 *               each an MSE mean over its embedding) == B reference calls at B=1.
 *  MEAN:        the reference called on a [B,80,T] tensor (MSE mean over B*D). */
enum { AVC_REDUCE_INDEPENDENT = 0, AVC_REDUCE_MEAN = 1 };

typedef struct avc_ctx avc_ctx;

/* Number of fp32 values avc_create expects in `weights` for this config. */
size_t avc_se_weight_count(const avc_se_cfg* cfg);

/* Create a context on HIP device `device`.  `weights` is a HOST pointer to the
 * speaker encoder's parameters concatenated in state_dict order
 * (conv_bank.{i}.weight, conv_bank.{i}.bias, ..., output_layer.bias), fp32,
 * `n_weights` == avc_se_weight_count(cfg). */
int avc_create(int device, const avc_se_cfg* cfg, const float* weights, size_t n_weights,
               avc_ctx** out);

void avc_destroy(avc_ctx* ctx);

/* emb[B, c_out] = SpeakerEncoder(x[B, c_in, T]) (forward only, fp32). */
int avc_se_forward(avc_ctx* ctx, const float* x, int B, int T, float* emb, void* stream);

/* Embedding attack (attack_utils.py:51-86) on B utterances of T frames.
 *   vc_tgt, adv_tgt, ptb0 : [B, c_in, T] device fp32 (ptb0 = the N(0,1) draw of
 *                           attack_utils.py:68, made by the caller)
 *   out_adv               : [B, c_in, T] device fp32 = vc_tgt + eps*tanh(ptb)
 *   losses (optional)     : [n_iters, B] device fp32, per-iteration per-utterance loss
 *                           L = MSE(emb,tgt) - 0.1*MSE(emb,org) (before that step's update)
 *   grad0 (optional)      : [B, c_in, T] device fp32, d L / d ptb at iteration 0
 * Adam(lr=1e-3, betas=(0.9,0.999), eps=1e-8) as torch.optim.Adam defaults. */
/* Perturbation update.
 *  ADAM (default): the reference's update -- adv = vc + eps*tanh(ptb), torch.optim.Adam on ptb
 *                  (attack_utils.py:68-86).
 *  PGD  (opt-in) : the sign-gradient + eps-clamp update BASELINE.json's north_star describes:
 *                  adv = vc + delta, delta0 = eps*tanh(ptb0), delta <- clamp(delta - pgd_step *
 *                  sign(d loss / d delta), -eps, eps).  Not in the reference's attacks (its only
 *                  eps-clamp is the VSMask header optimiser, models/header_model.py:65): parity
 *                  of this mode is unpinned; grad0 then holds d loss / d delta. */
enum { AVC_UPDATE_ADAM = 0, AVC_UPDATE_PGD = 1 };

typedef struct avc_attack_opts {
    int32_t precision;   /* AVC_PREC_* */
    int32_t reduction;   /* AVC_REDUCE_* */
    int32_t use_graph;   /* 1 = replay a captured hipGraph per iteration (default) */
    float* losses;
    float* grad0;
    int32_t update;      /* AVC_UPDATE_* */
    float pgd_step;      /* PGD step size (> 0 when update == AVC_UPDATE_PGD) */
} avc_attack_opts;

int avc_emb_attack(avc_ctx* ctx, const float* vc_tgt, const float* adv_tgt, const float* ptb0,
                   int B, int T, float eps, int n_iters, float* out_adv,
                   const avc_attack_opts* opts, void* stream);

/* The same attack with the target embedding given: tgt_emb [B, c_out] device fp32 =
 * SpeakerEncoder(adv_tgt) for an adv_tgt of any length (avc_se_forward).  The reference embeds
 * adv_tgt on its own (attack_utils.py:74-75), so its length never has to match vc_tgt's. */
int avc_emb_attack_emb(avc_ctx* ctx, const float* vc_tgt, const float* tgt_emb, const float* ptb0,
                       int B, int T, float eps, int n_iters, float* out_adv,
                       const avc_attack_opts* opts, void* stream);

/* Embedding attack on a RAGGED batch: utterance b has lengths[b] frames (HOST int array of B), as real
 * utterances do (/root/reference/attack.py:41-56 loads each from its own wav; every length has its own
 * reflect padding, ceil-mode pooling and time-mean).  vc_tgt, ptb0, out_adv and opts->grad0 are packed
 * [80][lengths[b]] blocks in batch order (device fp32); tgt_emb [B, c_out] = SpeakerEncoder(adv_tgt_b),
 * each adv_tgt embedded at its own length (avc_se_forward).  Every SpeakerEncoder pass is ONE launch over
 * the whole batch with per-workgroup lengths and offsets: on the fused runtime-length kernels when every
 * length is in (64, 128] (config.yaml model; env AVC_RAGGED_FUSED=0: never), else on the long engine;
 * utterance b's result equals its own avc_emb_attack_emb on the same kernels bit for bit.
 * opts->reduction must be INDEPENDENT.
 * Replaces B calls of attack_utils.emb_attack (attack_utils.py:51-86), one per utterance. */
int avc_emb_attack_ragged(avc_ctx* ctx, const float* vc_tgt, const int* lengths, int B, const float* tgt_emb,
                          const float* ptb0, float eps, int n_iters, float* out_adv,
                          const avc_attack_opts* opts, void* stream);

/* ---- voice-conversion path: ContentEncoder + Decoder (e2e / feedback attacks) ----
 * ContentEncoder / Decoder hyper-parameters, config.yaml model.ContentEncoder /
 * model.Decoder (/root/reference/models.py:121-208, 346-435).  act: 0 = ReLU, 1 = LeakyReLU. */
typedef struct avc_vc_cfg {
    int32_t ce_c_in, ce_c_h, ce_c_out, ce_kernel_size;
    int32_t ce_bank_size, ce_bank_scale, ce_c_bank, ce_n_conv_blocks;
    int32_t ce_subsample[AVC_MAX_BLOCKS];
    int32_t ce_act;
    int32_t dec_c_in, dec_c_cond, dec_c_h, dec_c_out, dec_kernel_size, dec_n_conv_blocks;
    int32_t dec_upsample[AVC_MAX_BLOCKS];
    int32_t dec_act;
    int32_t dec_sn;    /* 1: spectral-norm Decoder (models.py:382); the weights are the weight_orig tensors */
} avc_vc_cfg;

/* Number of fp32 values avc_attach_vc expects: content_encoder.* then decoder.* parameters,
 * each in state_dict order (AdaInVC.state_dict() minus the speaker_encoder.* entries). */
size_t avc_vc_weight_count(const avc_vc_cfg* cfg);

/* Attach the ContentEncoder and Decoder of the same AdaInVC model to `ctx` (HOST weights).
 * The HIP path is the fused per-utterance engine: the ContentEncoder must have the
 * SpeakerEncoder engine's fused shape (c_in=80, c_h=c_bank=c_out=128, bank_scale=1,
 * bank_size<=8, odd kernel_size<=5, <=8 blocks, subsample 1|2) and the Decoder c_in =
 * c_cond = c_h = 128, c_out = 80, odd kernel_size <= 5, <= 8 blocks, upsample 1|2; the
 * SpeakerEncoder of ctx must be fused-capable too.  Fails (non-zero) otherwise. */
int avc_attach_vc(avc_ctx* ctx, const avc_vc_cfg* cfg, const float* weights, size_t n_weights);

/* Spectral-norm Decoder (cfg->dec_sn = 1; models.py:382 wraps every Decoder layer in
 * torch.nn.utils.spectral_norm, and the reference never calls .eval(), so each Decoder forward
 * runs one power iteration and divides the layer's weight by sigma, updating its weight_u /
 * weight_v buffers).  libavc does the same before every Decoder forward it runs (attacks:
 * the precomputed targets and each iteration; inference; avc_decoder).  The state is every
 * layer's u then v, layers in module order -- in_conv_layer, first_conv_layers.*,
 * second_conv_layers.*, conv_affine_layers.*, out_conv_layer -- as HOST floats:
 *   avc_sn_state_count  number of floats (0 when the attached Decoder has no spectral norm)
 *   avc_set_sn_state    load it (before a call; the reference module's buffers)
 *   avc_get_sn_state    read it back (after a call: the buffers' new values)
 * Both synchronise the ctx's stream.  Replaces the weight_u / weight_v updates of
 * torch/nn/utils/spectral_norm.py:compute_weight as the reference runs it (models.py:382). */
size_t avc_sn_state_count(avc_ctx* ctx);
int avc_set_sn_state(avc_ctx* ctx, const float* uv, size_t n);
int avc_get_sn_state(avc_ctx* ctx, float* uv, size_t n);
/* The same state as a DEVICE buffer of avc_sn_state_count floats, copied on `stream` (ordered with
 * the caller's other work on it, no synchronisation): set = 1 loads it, set = 0 stores it. */
int avc_sn_state_dev(avc_ctx* ctx, float* uv, size_t n, int set, void* stream);
/* The hook's mode, as the Decoder module's .training says (torch spectral_norm.py compute_weight):
 *   train = 1 (default): one power iteration per forward, u / v updated;
 *   train = 0 (eval)   : sigma = u . (W v) from the stored u / v, which stay unchanged.
 * Ordered on `stream` like the calls that follow it. */
int avc_set_sn_train(avc_ctx* ctx, int train, void* stream);

/* Frames of the Decoder output for T input frames (T -> ContentEncoder length -> x upsample). */
int avc_vc_out_frames(avc_ctx* ctx, int T);

/* out[B, 80, Tn] = AdaInVC.inference(src, tgt) = Decoder(ContentEncoder(src).mu,
 * SpeakerEncoder(tgt))  (models.py:472-489); src, tgt [B, 80, T]; fp32. */
int avc_inference(avc_ctx* ctx, const float* src, const float* tgt, int B, int T, float* out, void* stream);

/* out[B, 80, Tn(T_src)] = Decoder(ContentEncoder(src).mu, emb): src [B, 80, T_src], emb [B, c_out]
 * = SpeakerEncoder(tgt) for a tgt of any length (avc_se_forward). */
int avc_inference_emb(avc_ctx* ctx, const float* src, int B, int T_src, const float* emb, float* out,
                      void* stream);

/* ContentEncoder.forward (models.py:181-210): mu, log_sigma [B, c_out, Tce] (either may be NULL) of
 * x [B, c_in, T]; Tce = avc_content_frames(T).  fp32. */
int avc_content_encoder(avc_ctx* ctx, const float* x, int B, int T, float* mu, float* log_sigma, void* stream);
int avc_content_frames(avc_ctx* ctx, int T);

/* Decoder.forward (models.py:403-435): out [B, c_out, Tz * prod(upsample)] = Decoder(z [B, c_in, Tz],
 * cond [B, c_cond]).  fp32.  Runs on the VC attack workspace of the shape (B, Tz * prod(subsample)):
 * the first call at a new Tz builds it (buffers, plans, autotune -- a SpeakerEncoder workspace included,
 * cached like an attack's, avc_set_ws_cache), and it needs the fused or long engine (it fails under
 * AVC_ENGINE_LAYERED, like the e2e / fb attacks). */
int avc_decoder(avc_ctx* ctx, const float* z, int B, int Tz, const float* cond, float* out, void* stream);

/* End-to-end attack (attack_utils.py:7-48) and feedback attack (attack_utils.py:89-130):
 * same buffers and options as avc_emb_attack plus vc_src [B, c_in, T].  losses (optional)
 * [n_iters, B]: e2e MSE(dec, tgt_out) - 0.1 MSE(dec, org_out); fb MSE(SE(dec), tgt_emb) -
 * 0.1 MSE(SE(dec), org_emb), both before that step's update. */
int avc_e2e_attack(avc_ctx* ctx, const float* vc_src, const float* vc_tgt, const float* adv_tgt,
                   const float* ptb0, int B, int T, float eps, int n_iters, float* out_adv,
                   const avc_attack_opts* opts, void* stream);
int avc_fb_attack(avc_ctx* ctx, const float* vc_src, const float* vc_tgt, const float* adv_tgt,
                  const float* ptb0, int B, int T, float eps, int n_iters, float* out_adv,
                  const avc_attack_opts* opts, void* stream);

/* e2e / feedback attacks with independent lengths: vc_src [B, c_in, T_src]; vc_tgt, ptb0 and
 * out_adv [B, c_in, T]; tgt_emb [B, c_out] = SpeakerEncoder(adv_tgt) (any adv_tgt length).
 * The decoder output (and the e2e objective) has Tn(T_src) frames, as in the reference, where
 * inference(vc_src, .) takes its length from vc_src (models.py:472-489). */
int avc_e2e_attack_emb(avc_ctx* ctx, const float* vc_src, int T_src, const float* vc_tgt,
                       const float* tgt_emb, const float* ptb0, int B, int T, float eps, int n_iters,
                       float* out_adv, const avc_attack_opts* opts, void* stream);
int avc_fb_attack_emb(avc_ctx* ctx, const float* vc_src, int T_src, const float* vc_tgt,
                      const float* tgt_emb, const float* ptb0, int B, int T, float eps, int n_iters,
                      float* out_adv, const avc_attack_opts* opts, void* stream);

/* ---- VSMask PredictiveModel forward (models/predictive_model.py:53-110, BASELINE config 5) ----
 * Eval-mode inference (BatchNorm running statistics).  `weights` = HOST fp32 floating
 * tensors of PredictiveModel.state_dict() in order (num_batches_tracked excluded). */
typedef struct avc_pm avc_pm;
size_t avc_pm_weight_count(void);
int avc_pm_create(int device, const float* weights, size_t n_weights, avc_pm** out);
void avc_pm_destroy(avc_pm* pm);
/* output window size for an H x W input ([B,1,80,100] -> [B,1,95,63]); non-zero if too small */
int avc_pm_out_shape(int H, int W, int* Ho, int* Wo);
/* y[B,1,Ho,Wo] = PredictiveModel(x[B,1,H,W]); device pointers, enqueued on `stream` */
int avc_pm_forward(avc_pm* pm, const float* x, int B, int H, int W, float* y, void* stream);

/* One block of the network on its own: layer 0..6 = down_blocks.0..6 (DownSamplingBlock.forward,
 * models/predictive_model.py:28-29), 7..11 = up_blocks.0..4 (UpSamplingBlock.forward, 50-51; the final
 * tanh is PredictiveModel.forward's, not the block's).  x [B][Cin][H][W] -> y [B][C][Ho][Wo] (NCHW,
 * device); avc_pm_block_shape gives C, Ho, Wo (non-zero if the input is too small) and, if Cin is
 * non-NULL, the layer's input channel count.  avc_pm_block_forward fails unless Cin equals the layer's
 * (torch's Conv2d shape check: the kernel would otherwise read B*Cin_layer*H*W floats of x). */
int avc_pm_block_shape(avc_pm* pm, int layer, int H, int W, int* C, int* Ho, int* Wo, int* Cin);
int avc_pm_block_forward(avc_pm* pm, int layer, const float* x, int B, int Cin, int H, int W, float* y,
                         void* stream);

/* ---- VSMask protect loop (/root/reference/vsmask.py:160-213, utils/audio.py:77-116,
 * models/header_model.py:70-95) ----
 * avc_vsmask_protect replaces VSMask._protect_waveform between waveform_to_mel and
 * mel_to_waveform (vsmask.py:181-208):
 *   acc = mel; acc[..., :min(T, Th)] += header;
 *   for start in range(0, T - W, S): acc[..., start+W : start+W+Wo] += PM(mel[..., start:start+W]);
 *   out = mel + band_clamp(acc - mel)   (f < int(F*0.3): eps1; f < int(F*0.7): eps2; else eps3)
 * mel [B][F][T] (the 4-D [B,1,F,T] mel the loop indexes); header [F][Th] or NULL; out
 * [B][F][T], must not alias mel; all device pointers, enqueued on `stream`.  The reference
 * as shipped cannot run this loop (SURVEY.md 2 note A): its mel is 3-D and its predictor
 * emits 95 rows for an 80-row mel.  Settled as: 4-D mel, predictor rows [0, min(F, Ho))
 * added, rows beyond F dropped.  All windows predict from the UNPERTURBED mel (as the
 * reference), so they run as one batched PredictiveModel forward.  The handle's scratch
 * is reused by every call: use one stream per avc_pm handle. */
int avc_vsmask_windows(int T, int window_size, int future_step, int* n_windows);
int avc_vsmask_protect(avc_pm* pm, const float* mel, int B, int F, int T, const float* header, int Th,
                       int window_size, int future_step, float eps1, float eps2, float eps3, float* out,
                       void* stream);
/* UniversalPerturbationHeader.optimize (header_model.py:25-68) as train_header.py:46,77-80
 * drives it (torch Adam(lr, betas, eps) on the header): per iteration
 *   perturbed = clamp(source + header, -1, 1);
 *   loss = MSE(SE(perturbed), SE(target)) - lambda_param * MSE(SE(perturbed), SE(source));
 *   Adam step on the header; header = clamp(header, -epsilon, epsilon).
 * source / target [N][80][T] (the reference's [N,1,80,T] mels, whose 4-D shape the
 * SpeakerEncoder cannot take: settled as 3-D); header [80][T] device, in / out (T = the
 * header length: the reference's broadcast needs equal lengths).  losses [n_iters][N] per-source
 * loss terms (their mean is the reference's loss) or NULL.  Runs on ctx's SpeakerEncoder with
 * the fused / long engine; precision AVC_PREC_*. */
int avc_header_optimize(avc_ctx* ctx, const float* source, const float* target, int N, int T, float* header,
                        float epsilon, float lambda_param, float lr, float beta1, float beta2, float adam_eps,
                        int n_iters, int precision, float* losses, void* stream);

/* The same, continuing a torch Adam optimiser: exp_avg / exp_avg_sq [80][T] device (in: its
 * state before the call, out: after; both or neither), step0 = the steps it has taken (its
 * state["step"]; the bias corrections continue from step0 + 1).  The reference passes one
 * optimizer whose state carries across optimize() calls (header_model.py:25-68). */
int avc_header_optimize_state(avc_ctx* ctx, const float* source, const float* target, int N, int T, float* header,
                              float epsilon, float lambda_param, float lr, float beta1, float beta2, float adam_eps,
                              int n_iters, int precision, float* losses, float* exp_avg, float* exp_avg_sq,
                              int step0, void* stream);

/* MelSpectrogramConverter.apply_weighted_constraint (utils/audio.py:77-116): x [B][F][T] ->
 * out = clamp(x, -eps, eps) with eps1 on rows [0, int(F*0.3)), eps2 to int(F*0.7), eps3 above. */
int avc_vsmask_band_clamp(int device, const float* x, int B, int F, int T, float eps1, float eps2, float eps3,
                          float* out, void* stream);

/* UniversalPerturbationHeader.apply_header (header_model.py:70-95):
 * out = clamp(mel + header on frames [0, min(T, Th)), -1, 1). */
int avc_vsmask_apply_header(int device, const float* mel, int B, int F, int T, const float* header, int Th,
                            float* out, void* stream);

/* ---- Mel front / back end (data_utils.py:16-197) ----
 * The reference's preprocess section of config.yaml.  librosa (<= 0.9, the version the
 * reference's positional calls need) semantics: centered frames, periodic Hann(win_length)
 * zero-padded to n_fft, Slaney mel filters with Slaney area normalisation.  pad_mode 0 =
 * reflect (librosa 0.8 stft default), 1 = constant.  n_fft: power of two in [16, 4096]. */
typedef struct {
    int32_t sample_rate, n_fft, hop_length, win_length, n_mels;
    float preemph, ref_db, max_db;
    int32_t pad_mode;
    /* 0: data_utils.py (librosa, above).  1: utils/audio.py:8-76 MelSpectrogramConverter (the
     * VSMask converter; torchaudio semantics): MelSpectrogram power 2 with an HTK mel filter
     * bank (norm None, f_max = sample_rate // 2), log10(clamp(., 1e-5)); preemph must be 0,
     * ref_db / max_db unused, no mean / std; mel2wav through avc_dsp_ta_mel2wav only. */
    int32_t flavor;
} avc_dsp_cfg;
typedef struct avc_dsp avc_dsp;
int avc_dsp_create(int device, const avc_dsp_cfg* cfg, avc_dsp** out);
void avc_dsp_destroy(avc_dsp* dsp);
/* STFT frames of an n-sample signal: 1 + n / hop_length (-1 on a bad config) */
int avc_dsp_frames(const avc_dsp_cfg* cfg, int n_samples);
/* HOST outputs (no device needed): mel_basis [n_mels][n_fft/2+1] = librosa.filters.mel(sr,
 * n_fft, n_mels); inv_mel [n_fft/2+1][n_mels] = inv_mel_matrix (either may be NULL) */
int avc_dsp_mel_basis(const avc_dsp_cfg* cfg, float* mel_basis, float* inv_mel);
/* file2mel after load + trim: wav [B][L] (trimmed waveforms of equal length L) ->
 * mel [B][Tf][n_mels] (transpose 0, file2mel's layout) or [B][n_mels][Tf] (transpose 1, the
 * attacks' [B,80,T] input), Tf = avc_dsp_frames(L).  mean / std (device [n_mels], both or
 * neither) fold normalize() in. */
int avc_dsp_wav2mel(avc_dsp* dsp, const float* wav, int B, int L, const float* mean, const float* std,
                    int transpose, float* mel, void* stream);
/* mel2wav: mel in the same layouts (denormalize() folded in when mean / std are given) ->
 * wav [B][hop_length * (Tf - 1)]: inverse dB, inv_mel_matrix, n_iter Griffin-Lim
 * iterations (the reference uses 100), de-emphasis. */
int avc_dsp_mel2wav(avc_dsp* dsp, const float* mel, int B, int Tf, int transpose, const float* mean,
                    const float* std, int n_iter, float* wav, void* stream);
/* griffin_lim(spect [B][n_fft/2+1][Tf], hop, win, n_fft, n_iter) -> wav [B][hop_length * (Tf - 1)] */
int avc_dsp_griffin_lim(avc_dsp* dsp, const float* spect, int B, int Tf, int n_iter, float* wav, void* stream);
/* flavor-1 context: MelSpectrogramConverter.mel_to_waveform (utils/audio.py:59-75): mel [B][n_mels][Tf]
 * log10 mel -> pow(10, .) -> InverseMelScale (the least-squares / minimum-norm solution of
 * fb^T X = mel, relu) -> GriffinLim(power 2, n_iter, momentum) -> wav [B][hop_length * (Tf - 1)].
 * angles0: device [B][n_fft/2+1][Tf] complex64 initial phases (GriffinLim's rand_init draw,
 * torch.rand(complex64)), or NULL for rand_init=False (all ones).  momentum in [0, 1). */
int avc_dsp_ta_mel2wav(avc_dsp* dsp, const float* mel, int B, int Tf, int n_iter, float momentum,
                       const float* angles0, float* wav, void* stream);
/* Per-launch HIP-event profiling of a DSP context (bench.py's roofline): while enabled every
 * launch is bracketed by events on the call's stream (and synchronised); per kernel name the
 * launch count and device milliseconds accumulate.  Enabling clears the counters. */
int avc_dsp_set_profiling(avc_dsp* dsp, int enable);
int avc_dsp_profile_count(avc_dsp* dsp);
int avc_dsp_profile_kernel(avc_dsp* dsp, int i, char* name, int name_len, long* launches, double* total_ms);

/* Compute engine of a context.
 *  AUTO    (default): FUSED for T <= 128, LONG above, when the config allows; else LAYERED.
 *  LAYERED: one implicit-GEMM launch per Conv1d / dgrad over the whole batch, activations in HBM
 *           (any SpeakerEncoder config, any T).
 *  FUSED  : one workgroup per utterance runs the whole conv stack out of LDS (2-3 launches per
 *           iteration); needs c_in=80, c_h=c_bank=c_out=128, bank_scale=1, bank_size<=8, odd
 *           kernel_size<=5, <=8 conv blocks with subsample 1|2, and T<=128 (above: LONG).
 *  LONG   : the same per-utterance kernels family for any T: each layer runs over chunks of 128
 *           frames staged through LDS, activations in per-utterance global scratch (the engine
 *           for real 128-600-frame utterances; selectable at any T for cross-checks).
 * avc_set_engine fails (non-zero) if FUSED / LONG is requested for a config that cannot use it;
 * avc_get_engine returns the engine a call with T frames would run on. */
enum { AVC_ENGINE_AUTO = 0, AVC_ENGINE_LAYERED = 1, AVC_ENGINE_FUSED = 2, AVC_ENGINE_LONG = 3 };
int avc_set_engine(avc_ctx* ctx, int engine);
int avc_get_engine(avc_ctx* ctx, int T);

/* Per-launch HIP-event profiling (bench.py's roofline).  While enabled, the
 * attack loop runs without graph replay and brackets every kernel launch with
 * HIP events on the ctx's stream, accumulating per-kernel-name launch counts,
 * device milliseconds and algorithmic FLOPs (weight gradients excluded). */
int avc_set_profiling(avc_ctx* ctx, int enable);
/* average ms per profiled attack iteration and algorithmic FLOP per iteration */
int avc_get_profile(avc_ctx* ctx, double* ms_per_iter, double* gemm_flop_per_iter);
int avc_profile_kernel_count(avc_ctx* ctx);
int avc_profile_kernel(avc_ctx* ctx, int i, char* name, int name_len, long* launches, double* total_ms,
                       double* total_flop);

/* In-graph kernel timing: the hot kernels' launch durations as they run inside the captured
 * attack-loop graphs, with no profiler attached (each workgroup stamps the device wall clock at its
 * start and end; a launch spans the earliest start to the latest end).  enable = 1 resets and starts
 * recording (process-wide, on ctx's device); enable = 0 stops and writes, per kernel and precision in
 * the order se_fwd_fused, se_bwd_fused, lz_se_fwd, lz_se_bwd, lz_dec_fwd, lz_dec_bwd, dec_fwd_fused,
 * dec_bwd_fused, se_attack_fused (the persistent emb attack: one launch per call), each as <fp32> then
 * <bf16>, the average launch duration in microseconds into avg_us[18] and the launch count into
 * launches[18] (either may be NULL).  Synchronises the device. */
int avc_ktime(avc_ctx* ctx, int enable, double* avg_us, int64_t* launches);

/* Workspace cache of a context.  A context keeps the buffers, launch plans and captured hipGraphs
 * of the last few (B, T, engine) shapes it ran (6 by default; env AVC_WS_CACHE overrides), most
 * recently used first, so a call at a shape seen before neither synchronises, allocates, plans nor
 * captures (real data: length-bucketed batches, an adv_tgt embedded at its own length).  Counters
 * since avc_create (any pointer may be NULL):
 *   builds   workspaces allocated and planned for a new shape
 *   replans  a cached workspace re-planned because a call needed more iterations than it holds
 *   hits     calls served by a cached workspace as it was
 *   (the e2e / fb ContentEncoder / Decoder workspaces, keyed by (B, T, T_src), count in the same totals)
 *   captures hipGraphs captured (attack loops, header optimiser)
 *   evictions cached workspaces freed to make room */
int avc_ws_stats(avc_ctx* ctx, int64_t* builds, int64_t* replans, int64_t* hits, int64_t* captures,
                 int64_t* evictions);
int avc_set_ws_cache(avc_ctx* ctx, int n_shapes);

const char* avc_last_error(void);
const char* avc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* AVC_H */
