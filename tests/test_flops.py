"""The frame-roofline FLOP counter (depth_completion_amd/flops.py) reproduces SURVEY.md §8d's table for the
shapes that table derives exactly (C1: latent 96x96, 10 steps; C2/C3: 72x96, 50 steps)."""
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


def test_ensemble_scales_with_seeds():
    one, ten = frame_flops(54, 96, 50, 1), frame_flops(54, 96, 50, 10)
    assert abs(ten["per_frame"] - 10 * one["per_frame"]) < 1e-3 * ten["per_frame"]
