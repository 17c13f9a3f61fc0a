"""Merge pmc_fold.py outputs of one build into one JSON (their kernel
entries side by side): python3 profiles/pmc_merge.py a.json b.json ..."""
import json
import sys


def main():
    out = None
    for f in sys.argv[1:]:
        with open(f) as fp:
            d = json.load(fp)
        if out is None:
            out = d
            continue
        if d["build_id"] != out["build_id"]:
            sys.exit(f"{f}: build {d['build_id']} != {out['build_id']}")
        for k, v in d.items():
            if isinstance(v, dict):
                out[k] = v
        out["source"] += "; " + d["source"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
