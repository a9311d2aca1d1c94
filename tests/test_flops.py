"""The frame-roofline FLOP counter (depth_completion_amd/flops.py) reproduces SURVEY.md §8d's table for the
shapes that table derives exactly (C1: latent 96x96, 10 steps; C2/C3: 72x96, 50 steps), and states the C4 / C5
rows it uses instead of SURVEY's (test_c4_c5_rows)."""
import pytest

from depth_completion_amd.flops import frame_flops


@pytest.mark.parametrize("h,w,steps,seeds,ufwd,udgrad,dec,enc,frame", [
    (96, 96, 10, 1, 2.138, 2.758, 0.318, 0.275, 55.9),
    (72, 96, 50, 1, 1.487, 1.836, 0.239, 0.206, 190.4),
])
def test_survey_table(h, w, steps, seeds, ufwd, udgrad, dec, enc, frame):
    f = frame_flops(h, w, steps, seeds)
    for key, want in (("unet_fwd", ufwd), ("unet_dgrad", udgrad), ("taesd_dec", dec), ("taesd_enc", enc),
                      ("per_frame", frame)):
        # the table is rounded to 3 decimals: allow half a unit of its last digit
        assert abs(f[key] / 1e12 - want) <= 5e-4 + 1e-3 * want, (key, f[key] / 1e12, want)


# C4 / C5 (latents 28x96 and 54x96, not multiples of 8).  flops.py counts the UNet at the latent that is actually
# run, halving with ceil (the stride-2 convs: 28 -> 14 -> 7 -> 4, 54 -> 27 -> 14 -> 7) and with the same per-layer
# formulas that reproduce the C1 / C2 rows above exactly; the TAESD columns equal SURVEY's.  SURVEY section 8d's
# UNet columns for these two rows (C4 0.441 / 0.486, C5 0.954 / 1.125 -> 55.8 / 1221.8 TF per frame) are not
# reproduced by those formulas at any one latent: 0.441 lies between the 24x96 (0.418) and 28x96 (0.499) UNet
# forwards, and no mix of a pixel-linear and a token-quadratic (attention) term fits C4, C5 and C2 together.
# bench.py's roofline uses these rows (62.0 / 1341.2 TF): its C4 / C5 fractions therefore read 11 % / 10 % higher
# than SURVEY's per-frame figures would give for the same frames/s.
@pytest.mark.parametrize("h,w,steps,seeds,ufwd,udgrad,dec,enc,frame,survey", [
    (28, 96, 50, 1, 0.499, 0.552, 0.093, 0.080, 62.0, 55.8),
    (54, 96, 50, 10, 1.061, 1.257, 0.179, 0.155, 1341.2, 1221.8),
])
def test_c4_c5_rows(h, w, steps, seeds, ufwd, udgrad, dec, enc, frame, survey):
    f = frame_flops(h, w, steps, seeds)
    for key, want in (("unet_fwd", ufwd), ("unet_dgrad", udgrad), ("taesd_dec", dec), ("taesd_enc", enc),
                      ("per_frame", frame)):
        assert abs(f[key] / 1e12 - want) <= 5e-4 + 1e-3 * want, (key, f[key] / 1e12, want)
    # the whole difference to SURVEY's row is in its UNet columns (TAESD equal): per frame
    # seeds x steps x (delta fwd + delta dgrad)
    assert 1.05 < frame / survey < 1.12


def test_survey_unet_c4_between_shapes():
    """SURVEY's C4 UNet forward (0.441 TF) sits between the 24x96 and 28x96 counts (see test_c4_c5_rows)."""
    from depth_completion_amd.flops import unet_flops
    assert unet_flops(24, 96)[0] / 1e12 < 0.441 < unet_flops(28, 96)[0] / 1e12


def test_ensemble_scales_with_seeds():
    one, ten = frame_flops(54, 96, 50, 1), frame_flops(54, 96, 50, 10)
    assert abs(ten["per_frame"] - 10 * one["per_frame"]) < 1e-3 * ten["per_frame"]
