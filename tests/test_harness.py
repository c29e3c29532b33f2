"""CPU test of the drop-in harness's calling pattern (tools/dropin_harness.cpp, the
RenderImageParallelMain restatement bench.py and the drop-in GPU tests drive): with
RenderJob doing nothing (SPT_HARNESS_NOOP, no GPU call), thousands of back-to-back frames
must finish.  RenderJob takes its slot only when its thread starts (Renderer.hpp:242-255),
so a frame's final wait can end before a spawned thread has started; with one slot count
shared by all frames and reset per frame, such a thread straddling the reset left the
count off by one and a later frame's final wait never ended (round 6: the old harness hung
in 3 of 5 runs of 2 000 frames).  Each frame now has its own count."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "simplepathtracer_amd", "lib", "spt_dropin_harness")


@pytest.mark.parametrize("tc,frames", [(4, 3000), (8, 600)])
def test_harness_frames_never_hang(tc, frames):
    if not os.path.exists(EXE):
        pytest.skip("harness not built (make -C simplepathtracer_amd/csrc)")
    env = dict(os.environ, SPT_HARNESS_NOOP="1")
    r = subprocess.run([EXE, "/dev/null", "1200", "800", "100", "50", str(tc), "0", str(frames)], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-500:]
    assert f"frames={frames} " in r.stdout
