"""Teacher-forced Tacotron-2 decoder training step on libtt2 (SURVEY.md §8f rank 1, configs[4]).

``TacotronTrainer`` mirrors what the reference's training graph does per step for the decoder
slice — ``Tacotron.initialize(is_training=True)`` with TacoTrainingHelper, ``add_loss()`` and
``add_optimizer()`` (tacotron/models/tacotron.py:31-35, 683-986, 1002-1251), driven by
``tacotron/train.py``'s ``sess.run([step, loss, optimize])`` — on the C ABI's training context
(csrc/train.hip).  Data-parallel training keeps one process per GPU; the reference's CPU tower
mean of the gradients (tacotron.py:1194-1208) becomes one RCCL all-reduce of the flat gradient
buffer between backward and the clipped Adam update.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check
from .weights import memory_width


def learning_rate(step, hp):
    """Tacotron._learning_rate_decay (tacotron.py:1227-1251): exponential decay from
    tacotron_start_decay every tacotron_decay_steps by tacotron_decay_rate, clipped to
    [tacotron_final_learning_rate, tacotron_initial_learning_rate]."""
    init = hp.tacotron_initial_learning_rate
    if not hp.tacotron_decay_learning_rate:
        return init
    lr = init * hp.tacotron_decay_rate ** ((step - hp.tacotron_start_decay) / hp.tacotron_decay_steps)
    return min(max(lr, hp.tacotron_final_learning_rate), init)


def teacher_forcing_ratio(global_step, hp):
    """TacoTrainingHelper's teacher-forcing ratio (helpers.py:65, 113-118): 'constant' ->
    tacotron_teacher_forcing_ratio; 'scheduled' -> _teacher_forcing_ratio_decay (helpers.py:140-180):
    the initial ratio before tacotron_teacher_forcing_start_decay, then
    tf.train.exponential_decay(init, global_step - start_decay, decay_steps, decay_exp_rate)."""
    if hp.tacotron_teacher_forcing_mode not in ("constant", "scheduled"):
        raise ValueError("tacotron_teacher_forcing_mode must be 'constant' or 'scheduled'")  # tacotron.py:202
    if hp.tacotron_teacher_forcing_mode == "constant":
        return float(hp.tacotron_teacher_forcing_ratio)
    init = float(hp.tacotron_teacher_forcing_init_ratio)
    if global_step < hp.tacotron_teacher_forcing_start_decay:
        return init
    return init * hp.tacotron_teacher_forcing_decay_exp_rate ** (
        (global_step - hp.tacotron_teacher_forcing_start_decay) / hp.tacotron_teacher_forcing_decay_steps)


def draw_teacher_forcing(T_out, ratio, rng):
    """The per-step draw of TacoTrainingHelper.next_inputs (helpers.py:126-131): for every step
    t >= 1 one uniform u for the whole batch, target frame t-1 fed when u < ratio.  Returns the
    u8 feed_target [T_out] the library takes (entry 0 = the go frame, always 1).  TF's Philox
    stream cannot be reproduced, so the draw is injected like the dropout keep bits."""
    feed = (rng.random(T_out) < ratio).astype(np.uint8)
    feed[0] = 1
    return feed


_UNSET = object()


def train_config(hp, batch, max_T_in, max_T_out, emt_only=False, precision="fp32", postnet=True,
                 frontend=False, max_T_ref=None, n_emt=0, n_spk=0, style="gst"):
    lib = _lib.load_library()
    cfg = _lib.TrainConfig()
    lib.tt2_train_default_config(ctypes.byref(cfg), batch, max_T_in, max_T_out)
    if len(hp.prenet_layers) != 2 or hp.prenet_layers[0] != hp.prenet_layers[1]:
        raise NotImplementedError("prenet_layers must be two equal widths on this build")
    if hp.decoder_layers != 2:
        raise NotImplementedError("decoder_layers = 2 on this build")
    if hp.outputs_per_step < 1:
        raise ValueError("outputs_per_step must be >= 1")
    # r frames per decoder step (tacotron.py:322-324; helpers.py:78,129): T_out counts frames, the
    # prenet / zoneout masks and the teacher-forcing draw count decoder steps T_out / r
    cfg.outputs_per_step = int(hp.outputs_per_step)
    if hp.tacotron_teacher_forcing_mode not in ("constant", "scheduled"):
        raise ValueError("tacotron_teacher_forcing_mode must be 'constant' or 'scheduled'")
    if hp.predict_linear:
        raise NotImplementedError("predict_linear (CBHG linear loss) is not built in the training step")
    cfg.smoothing = 1 if hp.smoothing else 0        # attention.py:71-91,150 (training graph too)
    # style path of the front end (tacotron.py:236-308): 'gst' (hp.use_gst; False = the embeddings),
    # 'embed' (args.pretrained_emb_disc_all: the reference embeddings themselves), 'adain'
    if style not in ("gst", "embed", "adain"):
        raise ValueError("style must be 'gst', 'embed' or 'adain'")
    if style != "gst" and not frontend:
        raise ValueError("style paths other than GST live in the front end (frontend=True)")
    cfg.memory_dim = memory_width(hp, emt_only, style)
    cfg.num_mels = hp.num_mels
    cfg.prenet_units = hp.prenet_layers[0]
    cfg.decoder_lstm_units = hp.decoder_lstm_units
    cfg.attention_dim = hp.attention_dim
    cfg.attention_filters = hp.attention_filters
    cfg.attention_kernel = hp.attention_kernel[0]
    cfg.zoneout = hp.tacotron_zoneout_rate
    reg = hp.tacotron_reg_weight
    if hp.tacotron_scale_regularization:                      # tacotron.py:857-861
        reg *= 1.0 / (2 * hp.max_abs_value) if hp.symmetric_mels else 1.0 / hp.max_abs_value
    cfg.reg_weight = reg
    cfg.adam_beta1 = hp.tacotron_adam_beta1
    cfg.adam_beta2 = hp.tacotron_adam_beta2
    cfg.adam_epsilon = hp.tacotron_adam_epsilon
    cfg.clip_norm = 1.0 if hp.tacotron_clip_gradients else 0.0
    cfg.mask_decoder = 1 if hp.mask_decoder else 0                    # tacotron.py:758-767
    cfg.pos_weight = float(hp.cross_entropy_pos_weight)               # modules.py:570
    if precision not in ("fp32", "bf16"):
        raise ValueError("precision must be 'fp32' or 'bf16'")
    cfg.precision = 1 if precision == "bf16" else 0
    # T2_output_range (tacotron.py:360-361): symmetric (-max, max), else (0, max)
    lo, hi = ((-hp.max_abs_value, hp.max_abs_value) if hp.symmetric_mels
              else (0.0, hp.max_abs_value))
    cfg.clip_outputs = 1 if hp.clip_outputs else 0
    cfg.clip_lo = lo - hp.lower_bound_decay
    cfg.clip_hi = hi
    # Postnet + after loss (tacotron.py:362-381, 775-776)
    cfg.postnet = 1 if postnet else 0
    cfg.postnet_layers = hp.postnet_num_layers
    cfg.postnet_channels = hp.postnet_channels
    cfg.postnet_kernel = hp.postnet_kernel_size[0]
    # front end (encoder + reference encoders + GST, tacotron.py:215-308)
    cfg.frontend = 1 if frontend else 0
    if frontend:
        from tacotron.utils.symbols import symbols
        cfg.n_symbols = len(symbols)
        cfg.embedding_dim = hp.embedding_dim
        cfg.enc_conv_layers = hp.enc_conv_num_layers
        cfg.enc_conv_kernel = hp.enc_conv_kernel_size[0]
        cfg.enc_conv_channels = hp.enc_conv_channels
        cfg.encoder_lstm_units = hp.encoder_lstm_units
        cfg.emt_only = 1 if emt_only else 0
        # hp.use_gst = False: the reference embeddings are the style embeddings (tacotron.py:284-291)
        cfg.use_gst = 1 if hp.use_gst and style == "gst" else 0
        cfg.adain = 1 if style == "adain" else 0
        cfg.num_gst = hp.num_gst
        cfg.num_heads = hp.num_heads
        cfg.style_embed_depth = hp.style_embed_depth
        cfg.style_att_dim = hp.style_att_dim
        cfg.reference_depth = hp.reference_depth
        for i, f in enumerate(hp.reference_filters):
            cfg.reference_filters[i] = f
        cfg.max_T_ref = max_T_ref or max_T_out
        # style-embedding losses of the default training graph (tacotron.py:486-495, 812-846): the
        # classifiers need the class counts (feeder.total_emt / total_spk); the orthogonality loss
        # needs both reference encoders
        # (neither is part of the adain / pretrained_emb_disc_all graphs: tacotron.py:485-495, 581, 841)
        if hp.tacotron_use_style_emb_disc and style == "gst":
            cfg.n_emt = int(n_emt)
            cfg.n_spk = 0 if emt_only else int(n_spk)
        if hp.tacotron_use_orthog_loss and not emt_only and style == "gst":
            cfg.orthog_weight = 0.02
    return cfg


def init_style_disc_weights(hp, n_emt, n_spk, emt_only=False, seed=None):
    """Fresh Style_Emb_Disc variables (tf.layers.dense: glorot-uniform kernel, zero bias) for
    the classes of this dataset, as TF initialises them at the start of training."""
    rng = np.random.default_rng(hp.tacotron_random_seed if seed is None else seed)
    W = {}
    for tag, n in (("emt", n_emt),) + ((() if emt_only else (("spk", n_spk),))):
        if n:
            lim = np.sqrt(6.0 / (128 + n))
            W["Tacotron_model/inference/style_disc_{}/dense/kernel".format(tag)] = \
                rng.uniform(-lim, lim, (128, n)).astype(np.float32)
            W["Tacotron_model/inference/style_disc_{}/dense/bias".format(tag)] = np.zeros(n, np.float32)
    return W


class TacotronTrainer(object):
    """One tt2_train_ctx on one GPU.  Inputs may be numpy arrays or torch tensors; everything
    runs on the trainer's own torch stream (passed to the library explicitly)."""

    def __init__(self, hp, weights, batch, max_T_in, max_T_out, device=0, emt_only=False,
                 precision="fp32", postnet=True, frontend=False, max_T_ref=None, tf_seed=None,
                 n_emt=0, n_spk=0, style="gst"):
        """n_emt / n_spk: classes of the style-embedding classifiers (frontend, when
        hp.tacotron_use_style_emb_disc); their variables are taken from ``weights`` or freshly
        initialised (init_style_disc_weights), and set_style_labels() feeds the labels."""
        import torch
        self.torch = torch
        self.lib = _lib.load_library()
        self.hp = hp
        self.device = torch.device("cuda", device)
        self.cfg = train_config(hp, batch, max_T_in, max_T_out, emt_only, precision, postnet, frontend,
                                max_T_ref, n_emt if frontend else 0, n_spk if frontend else 0, style)
        self.style = style
        # the Style_Emb_Disc variables this context trains, with the values it starts from (the
        # caller's, else a fresh draw): callers that save checkpoints merge them into their weights
        self.style_disc_weights = {}
        if self.cfg.n_emt or self.cfg.n_spk:
            fresh = init_style_disc_weights(hp, self.cfg.n_emt, self.cfg.n_spk, emt_only)
            weights = dict(weights)
            for k, v in fresh.items():
                weights.setdefault(k, v)
                self.style_disc_weights[k] = weights[k]
        self.frontend = frontend
        self.postnet = postnet
        self.B = batch
        self.r = int(hp.outputs_per_step)
        h = ctypes.c_void_p()
        check(self.lib.tt2_train_create(ctypes.byref(self.cfg), device, ctypes.byref(h)))
        self.h = h
        for name, arr in weights.items():
            if name.startswith("Tacotron_model/"):
                _lib.load_tensor(self.lib.tt2_train_load_tensor, self.h, name, arr)
        check(self.lib.tt2_train_finalize(self.h))
        self.stream = torch.cuda.Stream(device=self.device)
        n = ctypes.c_int64()
        check(self.lib.tt2_train_bind_grads_dev(self.h, None, ctypes.byref(n)))
        self.n_params = n.value
        self.grad_buf = None
        # Bind the flat gradient buffer before any backward pass: forward_backward() writes the
        # gradients wherever the context points, so binding it lazily in allreduce_grads() would
        # leave the first step's gradients in the library's own buffer and all-reduce zeros.
        self.bind_grad_buffer()
        self.global_step = 0
        self._keep = None
        # teacher forcing: drawn per step from the ratio schedule (TacoTrainingHelper) unless the
        # caller injects the draw through set_step_inputs(feed_target=...)
        self._feed_explicit = False
        # each data-parallel rank is its own tower and draws its own feed pattern (the reference's
        # towers draw independently): the rank joins the seed once torch.distributed is up
        seed = hp.tacotron_random_seed if tf_seed is None else tf_seed
        dist = torch.distributed
        rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self._tf_rng = np.random.default_rng([int(seed), rank] if rank else int(seed))
        self.ratio = None

    def close(self):
        if getattr(self, "h", None):
            self.lib.tt2_train_destroy(self.h)
            self.h = None

    __del__ = close

    def bind_grad_buffer(self):
        """Flat gradient buffer as a torch tensor (for RCCL all-reduce); returned view."""
        if self.grad_buf is None:
            # allocated (and zero-filled) on the trainer's stream, so the fill is ordered before
            # the library's first use of the buffer on that stream
            with self.torch.cuda.stream(self.stream):
                self.grad_buf = self.torch.zeros(self.n_params, dtype=self.torch.float32,
                                                 device=self.device)
            check(self.lib.tt2_train_bind_grads_dev(self.h, ctypes.c_void_p(self.grad_buf.data_ptr()),
                                                    None))
        return self.grad_buf

    def _dev(self, a, dtype):
        t = self.torch
        if a is None:
            return None
        if isinstance(a, t.Tensor):
            return a.to(self.device, dtype).contiguous()
        return t.from_numpy(np.ascontiguousarray(a)).to(self.device, dtype, non_blocking=False)

    def set_step_inputs(self, targets_lengths=_UNSET, feed_target=_UNSET):
        """Per-step inputs of the reference's training graph beyond the tensors; an argument left
        out keeps its current setting.  targets_lengths [B] (mask_decoder's loss masks,
        tacotron.py:56,758-767; required when hp.mask_decoder; None clears them).  feed_target
        [T_out / r] u8 (one per decoder step) injects the teacher-forcing draw (draw_teacher_forcing) for this and later
        steps; None = every step teacher-forced; auto_teacher_forcing() returns to drawing from
        the ratio schedule, which is the default."""
        if targets_lengths is not _UNSET:
            if targets_lengths is None:
                check(self.lib.tt2_train_set_target_lengths(self.h, None))
            else:
                tl = np.ascontiguousarray(np.asarray(targets_lengths, np.int32))
                if tl.shape != (self.B,):
                    raise ValueError("targets_lengths must be [batch]")
                check(self.lib.tt2_train_set_target_lengths(self.h, tl.ctypes.data_as(ctypes.c_void_p)))
        if feed_target is not _UNSET:
            self._feed_explicit = True
            self._set_feed(feed_target)

    def set_style_labels(self, emt_labels, spk_labels=None):
        """Emotion / speaker labels [B] of this step's references (the style-embedding
        classifiers' targets, feeder.emt_labels / spk_labels); None, None clears them."""
        if emt_labels is None and spk_labels is None:
            check(self.lib.tt2_train_set_style_labels(self.h, None, None))
            return
        e = np.ascontiguousarray(np.asarray(emt_labels, np.int32).reshape(-1))
        sp = None if spk_labels is None else np.ascontiguousarray(np.asarray(spk_labels, np.int32).reshape(-1))
        if e.shape != (self.B,) or (sp is not None and sp.shape != (self.B,)):
            raise ValueError("labels must be [batch]")
        check(self.lib.tt2_train_set_style_labels(self.h, e.ctypes.data_as(ctypes.c_void_p),
                                                  None if sp is None else sp.ctypes.data_as(ctypes.c_void_p)))

    def auto_teacher_forcing(self):
        """Draw the teacher forcing per step from the ratio schedule again (the default)."""
        self._feed_explicit = False

    def _set_feed(self, feed_target):
        if feed_target is None:
            check(self.lib.tt2_train_set_teacher_forcing(self.h, None, 0))
        else:
            ft = np.ascontiguousarray(np.asarray(feed_target, np.uint8))
            check(self.lib.tt2_train_set_teacher_forcing(self.h, ft.ctypes.data_as(ctypes.c_void_p),
                                                         int(ft.shape[0])))

    def _teacher_forcing(self, T_out):
        """TacoTrainingHelper (helpers.py:99-131): the ratio of this step -- the schedule at the
        global step BEFORE this step's update, as TF reads the variable -- and one uniform draw
        per decoder step from the trainer's seeded generator (TF's Philox stream cannot be
        reproduced).  A ratio >= 1 feeds every target frame and draws nothing."""
        if self._feed_explicit:
            return
        self.ratio = teacher_forcing_ratio(self.global_step, self.hp)
        self._set_feed(None if self.ratio >= 1.0 else
                       draw_teacher_forcing(T_out // self.r, self.ratio, self._tf_rng))

    def _steps(self, T_out):
        """Decoder steps of a T_out-frame batch (the feeder pads targets to a multiple of r,
        feeder.py:283-310)."""
        if T_out % self.r:
            raise ValueError("T_out = {} is not a multiple of outputs_per_step = {}".format(T_out, self.r))
        return T_out // self.r

    def forward_backward(self, memory, lengths, targets, stop_targets, prenet_masks,
                         zoneout_masks=None, postnet_masks=None):
        """Teacher-forced forward + losses + backward; gradients land in the flat buffer.
        targets [B, T_out, 80] / stop_targets [B, T_out] in frames; prenet_masks [T_dec, 2, B, P]
        and zoneout_masks [T_dec, 4, B, H] per decoder step (T_dec = T_out / outputs_per_step).
        postnet_masks: Postnet dropout keep bits [layers, B, T_out, channels] (None = no
        dropout).  Target lengths / teacher-forcing draw: set_step_inputs."""
        t = self.torch
        with t.cuda.stream(self.stream):
            mem = self._dev(memory, t.float32)
            lens = self._dev(lengths, t.int32)
            tg = self._dev(targets, t.float32)
            st = self._dev(stop_targets, t.float32)
            pm = self._dev(prenet_masks, t.uint8)
            zm = self._dev(zoneout_masks, t.uint8)
            pnm = self._dev(postnet_masks, t.uint8) if self.postnet else None
            B, T_in, _ = mem.shape
            T_out = tg.shape[1]
            T_dec = self._steps(T_out)
            if B != self.B:
                raise ValueError("batch {} != trainer batch {}".format(B, self.B))
            if tuple(pm.shape) != (T_dec, 2, B, self.cfg.prenet_units):
                raise ValueError("prenet_masks must be [T_out / r, 2, B, prenet_units]")
            self._teacher_forcing(T_out)
            if zm is not None and tuple(zm.shape) != (T_dec, 4, B, self.cfg.decoder_lstm_units):
                raise ValueError("zoneout_masks must be [T_out / r, 4, B, decoder_lstm_units]")
            if pnm is not None and tuple(pnm.shape) != (self.cfg.postnet_layers, B, T_out,
                                                        self.cfg.postnet_channels):
                raise ValueError("postnet_masks must be [layers, B, T_out, channels]")
            self._keep = (mem, lens, tg, st, pm, zm, pnm)  # alive until the stream has used them
            ptr = (lambda x: None if x is None else ctypes.c_void_p(x.data_ptr()))
            check(self.lib.tt2_train_forward_backward_dev(
                self.h, ptr(mem), ptr(lens), ptr(tg), ptr(st), ptr(pm), ptr(zm), ptr(pnm), T_in, T_out,
                ctypes.c_void_p(self.stream.cuda_stream)))

    def forward_backward_text(self, ids, lengths, ref_emt, ref_spk, targets, stop_targets,
                              prenet_masks, zoneout_masks=None, postnet_masks=None,
                              enc_conv_masks=None, enc_zoneout_masks=None):
        """The whole configs[4] step (frontend context): ids [B,T_in] + lengths, reference mels
        [B,T_ref,80] -> encoder / reference encoders / GST in training mode -> decoder + Postnet ->
        backward through everything.  enc_conv_masks [layers,B,T_in,C] and enc_zoneout_masks
        [T_in,2,2,B,U] are keep bits (None = no conv dropout / inference zoneout mix)."""
        t = self.torch
        if not self.frontend:
            raise RuntimeError("trainer built without frontend=True")
        with t.cuda.stream(self.stream):
            ids_d = self._dev(ids, t.int32)
            lens = self._dev(lengths, t.int32)
            re = self._dev(ref_emt, t.float32)
            rs = self._dev(ref_spk, t.float32)
            tg = self._dev(targets, t.float32)
            st = self._dev(stop_targets, t.float32)
            pm = self._dev(prenet_masks, t.uint8)
            zm = self._dev(zoneout_masks, t.uint8)
            pnm = self._dev(postnet_masks, t.uint8) if self.postnet else None
            em = self._dev(enc_conv_masks, t.uint8)
            ezm = self._dev(enc_zoneout_masks, t.uint8)
            B, T_in = ids_d.shape
            T_out = tg.shape[1]
            T_dec = self._steps(T_out)
            T_ref = re.shape[1]
            if B != self.B:
                raise ValueError("batch {} != trainer batch {}".format(B, self.B))
            if rs is not None and tuple(rs.shape) != tuple(re.shape):
                raise ValueError("ref_emt and ref_spk must have the same shape")
            if tuple(pm.shape) != (T_dec, 2, B, self.cfg.prenet_units):
                raise ValueError("prenet_masks must be [T_out / r, 2, B, prenet_units]")
            if zm is not None and tuple(zm.shape) != (T_dec, 4, B, self.cfg.decoder_lstm_units):
                raise ValueError("zoneout_masks must be [T_out / r, 4, B, decoder_lstm_units]")
            self._teacher_forcing(T_out)
            if em is not None and tuple(em.shape) != (self.cfg.enc_conv_layers, B, T_in,
                                                      self.cfg.enc_conv_channels):
                raise ValueError("enc_conv_masks must be [layers, B, T_in, channels]")
            if ezm is not None and tuple(ezm.shape) != (T_in, 2, 2, B, self.cfg.encoder_lstm_units):
                raise ValueError("enc_zoneout_masks must be [T_in, 2, 2, B, encoder_lstm_units]")
            self._keep = (ids_d, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
            ptr = (lambda x: None if x is None else ctypes.c_void_p(x.data_ptr()))
            check(self.lib.tt2_train_forward_backward_text_dev(
                self.h, ptr(ids_d), ptr(lens), ptr(re), ptr(rs), T_ref, ptr(tg), ptr(st), ptr(pm),
                ptr(zm), ptr(pnm), ptr(em), ptr(ezm), T_in, T_out,
                ctypes.c_void_p(self.stream.cuda_stream)))

    def allreduce_grads(self, group=None):
        """Tower mean (tacotron.py:1194-1208) as one all-reduce over the flat gradient buffer."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return
        from .parallel import tower_mean_
        buf = self.bind_grad_buffer()
        with self.torch.cuda.stream(self.stream):
            tower_mean_(buf, group)

    def _stats(self):
        """Every BN moving_mean / moving_variance packed into one device buffer (library order)."""
        n = ctypes.c_int64()
        check(self.lib.tt2_train_moving_stats_dev(self.h, None, ctypes.byref(n), 0, None))
        if n.value == 0:
            return None
        with self.torch.cuda.stream(self.stream):
            buf = self.torch.empty(n.value, dtype=self.torch.float32, device=self.device)
            check(self.lib.tt2_train_moving_stats_dev(self.h, ctypes.c_void_p(buf.data_ptr()), None, 0,
                                                      ctypes.c_void_p(self.stream.cuda_stream)))
        return buf

    def sync_moving_stats(self, before=None, group=None):
        """Make every rank's batch-norm moving statistics the reference's single shared set.

        In the reference all towers run the UPDATE_OPS of ONE set of moving-statistics variables
        (tacotron.py:1088-1090 inside the tower loop 1194-1208): the towers' updates
        m <- mu·m + (1-mu)·x_k compose one after another.  Here each rank applied its own update
        in apply(); with ``before`` (the packed statistics before that apply, as step() passes
        them) the ranks rebuild the composition in rank order with one SUM all-reduce:
        m_N = mu^N·m_0 + Σ_k mu^(N-1-k)·(m_k - mu·m_0), where m_k is rank k's own update.  TF runs
        the towers' ops in an unspecified order; rank order is one of the orders it may take.
        Without ``before`` the ranks keep the mean of their updates (order-free, not exactly any
        of TF's orders).  Stream-ordered: no host synchronisation."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
            return
        from .parallel import all_reduce_sum_, tower_mean_
        buf = self._stats()
        if buf is None:
            return
        N, k = dist.get_world_size(group), dist.get_rank(group)
        mu = float(self.cfg.bn_momentum)
        with self.torch.cuda.stream(self.stream):
            if before is None:
                tower_mean_(buf, group)
            else:
                buf.sub_(before, alpha=mu).mul_(mu ** (N - 1 - k))
                all_reduce_sum_(buf, group)
                buf.add_(before, alpha=mu ** N)
            check(self.lib.tt2_train_moving_stats_dev(self.h, ctypes.c_void_p(buf.data_ptr()), None, 1,
                                                      ctypes.c_void_p(self.stream.cuda_stream)))
        self._stats_keep = (buf, before)  # alive until the stream has consumed them

    def apply(self, global_step=None, lr=None):
        """clip_by_global_norm(1.0) + Adam at update count ``global_step`` (1-based).

        The learning rate is the schedule at ``global_step - 1``: TF's apply_gradients reads the
        global_step variable before incrementing it (tacotron.py:1029 passes it to
        _learning_rate_decay, evaluated in the same session.run), so the first update uses
        step 0.  Adam's bias correction counts updates, i.e. ``global_step``."""
        if global_step is None:
            global_step = self.global_step + 1
        self.global_step = global_step
        if lr is None:
            lr = learning_rate(global_step - 1, self.hp)
        check(self.lib.tt2_train_apply_dev(self.h, float(lr), int(global_step),
                                           ctypes.c_void_p(self.stream.cuda_stream)))
        return lr

    def step(self, memory, lengths, targets, stop_targets, prenet_masks, zoneout_masks=None,
             postnet_masks=None):
        """One training step (forward, backward, DP all-reduce when initialised, clipped Adam);
        returns the losses dict."""
        self.forward_backward(memory, lengths, targets, stop_targets, prenet_masks, zoneout_masks,
                              postnet_masks)
        return self.optimizer_step()

    def step_text(self, *args, **kwargs):
        """The whole configs[4] step: forward_backward_text(*args, **kwargs), then
        optimizer_step(); returns the losses dict."""
        self.forward_backward_text(*args, **kwargs)
        return self.optimizer_step()

    def optimizer_step(self, global_step=None):
        """After a forward_backward: DP all-reduce (when initialised), clipped Adam at
        ``global_step`` (default: the next update), BN moving statistics composed over ranks;
        returns the losses dict."""
        self.allreduce_grads()
        import torch.distributed as dist
        dp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        before = self._stats() if dp else None
        self.apply(global_step)
        if dp:
            self.sync_moving_stats(before)
        return self.losses()

    def losses(self):
        out = np.zeros(5, np.float32)
        ms = ctypes.c_float()
        check(self.lib.tt2_train_losses(self.h, out.ctypes.data_as(ctypes.c_void_p),
                                        ctypes.byref(ms)))
        sl = np.zeros(3, np.float32)
        check(self.lib.tt2_train_style_losses(self.h, sl.ctypes.data_as(ctypes.c_void_p)))
        return dict(before=float(out[0]), stop_token=float(out[1]), regularization=float(out[2]),
                    after=float(out[4]), style_emb_loss_emt=float(sl[0]), style_emb_loss_spk=float(sl[1]),
                    style_emb_orthog_loss=float(sl[2]),
                    loss=float(out[0] + out[1] + out[2] + out[4] + sl[0] + sl[1] + sl[2]),
                    grad_norm=float(out[3]),
                    forward_backward_ms=float(ms.value))

    def get(self, name, which=0, shape=None):
        """which: 0 param, 1 gradient, 2 Adam m, 3 Adam v; name 'memory' = d loss / d memory."""
        if shape is None:
            raise ValueError("shape required")
        out = np.zeros(shape, np.float32)
        check(self.lib.tt2_train_get_tensor(self.h, name.encode(), which,
                                            out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def mel_outputs(self, T_out):
        """mel_outputs of the last forward (tacotron.py:375-378): clip(decoder_output + Postnet
        projection) [B, T_out, 80] (decoder_output alone without the Postnet)."""
        fr, _, _ = self.outputs(None, T_out)
        if not self.postnet:
            return fr
        x = fr + self.get("postnet:projection", 0, fr.shape)
        return np.clip(x, self.cfg.clip_lo, self.cfg.clip_hi) if self.cfg.clip_outputs else x

    def outputs(self, T_in, T_out):
        """The last forward's frames [B, T_out, 80], stop logits [B, T_out] and (T_in given)
        alignments [B, T_in, T_out / r] (one per decoder step)."""
        fr = np.zeros((self.B, T_out, self.cfg.num_mels), np.float32)
        st = np.zeros((self.B, T_out), np.float32)
        al = None if T_in is None else np.zeros((self.B, T_in, self._steps(T_out)), np.float32)
        check(self.lib.tt2_train_outputs(self.h, fr.ctypes.data_as(ctypes.c_void_p),
                                         st.ctypes.data_as(ctypes.c_void_p),
                                         None if al is None else al.ctypes.data_as(ctypes.c_void_p)))
        return fr, st, al
