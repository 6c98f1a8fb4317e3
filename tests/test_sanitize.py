"""The oracle's C++ under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md §5): oracle/sanitize_check.cpp calls every oracle entry point on a
synthetic frame pair and on the edge cases (tiny / blank frames, empty
descriptor sets, < 5 correspondences, k above the train count); any sanitizer
report aborts it with a non-zero status."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_is_clean_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "build", "sanitize_check")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
    assert "0 failed checks" in r.stdout
