"""ASan + UBSan build of the C++ grammar engine, random-walk fuzzed over the real intent grammar
(sanitizers on the native runtime; GPU sanitizers are unavailable on this pool)."""
import os
import shutil
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan")
def test_grammar_engine_asan_ubsan_fuzz(capsys):
    import sanitize_native

    # seed 1 / 30 walks / 20k tokens reproduces the REC-count cache-key collision fixed in grammar.cpp
    rc = sanitize_native.main(["--walks", "30", "--budget", "512", "--vocab-limit", "20000", "--seed", "1"])
    out = capsys.readouterr().out
    assert rc == 0 and "FUZZ_OK" in out, out
