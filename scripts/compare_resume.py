"""Compare the logged losses of an uninterrupted fine-tune with a checkpoint + resume run.
usage: python scripts/compare_resume.py full.jsonl part1.jsonl part2.jsonl"""
import json
import sys


def load(p):
    out = {}
    for line in open(p):
        r = json.loads(line)
        if "loss" in r and "step" in r:
            out[int(r["step"])] = float(r["loss"])
    return out


def final(p):
    """(bit-sum, weighted bit-sum) of the final fp32 master weights, when the run logged them."""
    for line in open(p):
        r = json.loads(line)
        if r.get("kind") == "final":
            return (r["master_bits_sum"], r["master_bits_wsum"])
    return None


def main():
    full, p1, p2 = (load(p) for p in sys.argv[1:4])
    resumed = {**p1, **p2}  # steps logged again after the resume (150..159) come from the resumed run
    steps = sorted(set(full) & set(resumed))
    worst = 0.0
    for s in steps:
        d = abs(full[s] - resumed[s])
        worst = max(worst, d)
        print(f"step {s:4d}  uninterrupted {full[s]:.5f}  resumed {resumed[s]:.5f}  |diff| {d:.2e}")
    first, last = min(full), max(full)
    bitwise = all(full[s] == resumed[s] for s in steps)
    print(f"loss {full[first]:.4f} (step {first}) -> {full[last]:.4f} (step {last}); "
          f"max |uninterrupted - resumed| over {len(steps)} logged steps: {worst:.3e}; "
          f"bitwise equal at every logged step: {bitwise}")
    fa, fb = final(sys.argv[1]), final(sys.argv[3])
    if fa is not None and fb is not None:
        same = fa == fb
        print(f"final fp32 master digest: {fa} vs {fb} -> {'IDENTICAL' if same else 'DIFFERENT'}")


if __name__ == "__main__":
    main()
