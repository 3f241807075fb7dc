"""ExtractConfig's default model-stream count follows the hardware queues the
process has (package HW_QUEUES from GPU_MAX_HW_QUEUES; ADVICE r4 / VERDICT r4
item 7).  CPU only."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_default_model_streams_by_queue_count(mdx):
    from moseq2_detectron_extract_amd.pipeline import default_model_streams
    assert default_model_streams(8) == 4
    assert default_model_streams(4) == 2
    assert default_model_streams(3) == 1
    assert default_model_streams(1) == 1
    assert default_model_streams(10) == 6
    assert default_model_streams(12) == 8
    assert default_model_streams(32) == 8


def _probe(env):
    code = ("import sys; sys.path.insert(0, %r); import mdx_pkg; m = mdx_pkg.load(); import os; "
            "from moseq2_detectron_extract_amd.pipeline import ExtractConfig; "
            "print(m.HW_QUEUES, os.environ.get('GPU_MAX_HW_QUEUES'), ExtractConfig().model_streams)" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.split()


def test_package_sets_queues_before_hip_starts():
    """Unset: the package sets 12 queues before HIP initialises and the
    extractor runs 8 forwards; a caller's own setting is kept."""
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    assert _probe(env) == ["12", "12", "8"]
    assert _probe(dict(env, GPU_MAX_HW_QUEUES="8")) == ["8", "8", "4"]
    assert _probe(dict(env, GPU_MAX_HW_QUEUES="4")) == ["4", "4", "2"]
