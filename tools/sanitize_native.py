"""Build the C++ grammar engine with AddressSanitizer + UndefinedBehaviorSanitizer (host code only)
and run the random-walk fuzz driver (csrc/runtime/tests/grammar_fuzz.cpp) on the real intent
grammar and the Llama-3 vocabulary.  GPU sanitizers are not available on this pool; the kernels
are covered by the numerics suite instead.

    python tools/sanitize_native.py [--walks 40] [--budget 400]
"""
import argparse
import os
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--walks", type=int, default=40)
    ap.add_argument("--budget", type=int, default=400)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--vocab-limit", type=int, default=0, help="use only the first N tokens (+ eos) for speed")
    args = ap.parse_args(argv)
    from voice_enabled_browser_automation_amd.grammar import ir_from_json_schema, parse_response_schema
    from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer

    tok = load_tokenizer("llama3")
    tb = tok.token_bytes()
    eos = {tok.token_to_id("<|eot_id|>"), tok.token_to_id("<|end_of_text|>")}
    ids = list(range(len(tb)))
    if args.vocab_limit:
        ids = list(range(args.vocab_limit))
    with tempfile.TemporaryDirectory() as d:
        ir = os.path.join(d, "ir.json")
        with open(ir, "w") as f:
            f.write(ir_from_json_schema(parse_response_schema()))
        vb = os.path.join(d, "vocab.bin")
        with open(vb, "wb") as f:
            toks = [b"" if i in eos else (tb[i] or b"\xff\xfe") for i in ids] + [b""]  # last: eos
            f.write(struct.pack("<I", len(toks)))
            for t in toks:
                f.write(struct.pack("<I", len(t)) + t)
        exe = os.path.join(d, "grammar_fuzz")
        src = [os.path.join(ROOT, "csrc", "runtime", "grammar.cpp"),
               os.path.join(ROOT, "csrc", "runtime", "tests", "grammar_fuzz.cpp")]
        cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
               "-fno-sanitize-recover=undefined", "-o", exe] + src
        subprocess.run(cmd, check=True)
        # verify_asan_link_order=0: the environment may preload other libraries ahead of the runtime
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
                   UBSAN_OPTIONS="print_stacktrace=1")
        r = subprocess.run([exe, ir, vb, str(args.walks), str(args.budget), str(args.seed)], env=env,
                           capture_output=True, text=True)
        sys.stdout.write(r.stdout)
        sys.stderr.write(r.stderr[-4000:])
        return r.returncode


if __name__ == "__main__":
    sys.exit(main())
