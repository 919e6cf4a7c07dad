"""Summarise a cProfile dump (bench.py with DXA_BENCH_CPROFILE=path): top own-time functions, top cumulative, and
the callers of the host-synchronising / allocating / launching primitives.
    python tools/pstats_report.py path.prof [steps]"""
import io
import pstats
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    print(f"# {path}: {steps} timed steps")
    for key, n in (("tottime", 50), ("cumulative", 70)):
        s = io.StringIO()
        pstats.Stats(path, stream=s).sort_stats(key).print_stats(n)
        print(f"==== by {key}")
        print("\n".join(l for l in s.getvalue().splitlines() if l.strip()))
    for pat in ("tolist", "'item'", "torch.empty", "native.py.*call", "acquire", "synchronize", "to' of"):
        s = io.StringIO()
        st = pstats.Stats(path, stream=s)
        st.sort_stats("tottime").print_callers(pat, 25)
        print(f"==== callers of {pat}")
        print("\n".join(l for l in s.getvalue().splitlines() if l.strip())[-6000:])


if __name__ == "__main__":
    main()
