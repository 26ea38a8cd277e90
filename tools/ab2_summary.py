"""Summary of tools/ab_variants.sh secondary runs: python tools/ab2_summary.py TAG variant..."""
import json
import sys

tag, vs = sys.argv[1], sys.argv[2:]
for r in (1, 2, 3):
    for v in vs:
        try:
            d = json.loads(open(f"gpurun_out/ab2_{tag}_{v}_{r}.json").read().splitlines()[-1])
        except OSError:
            continue
        rb = d.get("c2_randomized_batch", {}).get("by_sub_batch", {})
        lat = d.get("latency", {})
        c3 = d.get("c3_epoch", {})
        c5 = d.get("c5_multi_pairing", {}).get("batched", {})
        print(v, r, "C2", round(d["value"]),
              "rb64", round(rb.get("64", {}).get("clean", {}).get("verifications_per_s", 0)),
              "rb8t", round(rb.get("8", {}).get("tampered_1_in_16", {}).get("verifications_per_s", 0)),
              "lat", round(lat.get("bls_verify_ms", {}).get("median", 0), 3),
              "c3", round(c3.get("attestations_per_s", 0)),
              "c5", round(c5.get("pairings_per_s", 0)))
