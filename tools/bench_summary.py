"""Print the headline fields of a bench.py JSON line (the last line of a file)."""
import json
import sys


def main(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print("value %.4g %s  one_batch %s  ms/step %.4g  e2e %s" % (
        d["value"], d["unit"], "%.4g" % d["value_one_batch"] if "value_one_batch" in d else "-", d["ms_per_step"],
        "%.4g" % d["e2e"]["transitions_per_s"] if "e2e" in d else "-"))
    print("roofline %s frac %.3f kernel %.4g ms wait %s busy %s" % (
        r.get("bound"), r.get("frac", 0), r.get("kernel_avg_ms", 0), r.get("wait_any_frac"), r.get("busy_frac")))
    for k, v in (d.get("cfr_configs") or {}).items():
        if "error" in v:
            print(k, v["error"])
            continue
        cb = v.get("cpu_baseline") or {}
        print("config %s: %.4g %s (reps %s) carry/s %.3g  cpu %s" % (
            k, v["value"], v["unit"], [round(x, 1) for x in v["all_reps_value"]], v["carry_out_per_s"],
            "%.4g (1 core %.4g, %s cores)" % (cb["value"], cb["one_core"], cb["cores"]) if "value" in cb else cb))


if __name__ == "__main__":
    main(sys.argv[1])
