"""TEST INFRASTRUCTURE ONLY — adapters from an HParams object to the oracle's plain dicts."""


def oracle_hp(hp, synthesis_constraint=False, style="gst"):
    """style: 'gst' | 'embed' | 'adain' (tacotron.py:236-308); 'gst' without hp.use_gst is 'embed'."""
    return dict(style="embed" if style == "gst" and not hp.use_gst else style,
                zoneout=hp.tacotron_zoneout_rate, num_mels=hp.num_mels,
                max_abs_value=hp.max_abs_value, lower_bound_decay=hp.lower_bound_decay,
                clip_outputs=hp.clip_outputs, stop_at_any=hp.stop_at_any,
                mask_encoder=hp.mask_encoder, cumulative=hp.cumulative_weights,
                synthesis_constraint=synthesis_constraint,
                synthesis_constraint_type=hp.synthesis_constraint_type,
                attention_win_size=hp.attention_win_size, num_heads=hp.num_heads,
                smoothing=hp.smoothing)


def wavenet_oracle_hp(hp):
    return dict(layers=hp.layers, stacks=hp.stacks, residual_channels=hp.residual_channels,
                legacy=hp.legacy, residual_legacy=hp.residual_legacy,
                log_scale_min=hp.log_scale_min, upsample_scales=list(hp.upsample_scales),
                freq_axis_kernel_size=hp.freq_axis_kernel_size, max_abs_value=hp.max_abs_value,
                kernel_size=hp.kernel_size, upsample_type=hp.upsample_type,
                upsample_activation=hp.upsample_activation, leaky_alpha=hp.leaky_alpha,
                NN_init=hp.NN_init, log_scale_min_gauss=hp.log_scale_min_gauss,
                input_type=getattr(hp, "input_type", "raw"), quantize_channels=hp.quantize_channels)
