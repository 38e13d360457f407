"""SteppingDriver pull logic on the CPU (no GPU): tests/cpp/driver_logic.cpp drives host-memory
Source / Filter / Sink nodes through the ISteppingDriver ABI of libgpusdrpipeline.so and checks
the whole-stream results (reference SteppingDriver.cpp:102-366, count rule Fir.cpp:178-186)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stepping_driver_host_nodes():
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "cuda-sdr_amd")], check=True, timeout=900)
    cpp = os.path.join(REPO, "tests", "cpp")
    subprocess.run(["make", "-s", "-C", cpp, "_build/driver_logic"], check=True, timeout=300)
    r = subprocess.run([os.path.join(cpp, "_build", "driver_logic")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ALL PASS" in r.stdout, r.stdout + r.stderr
