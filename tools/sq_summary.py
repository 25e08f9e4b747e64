"""Per-kernel SQ counter summary of one rocprofv3 --pmc pass (tools/gpu_round.sh sq):
wave cycles split into busy / waiting, VALU and vector-memory instructions per wave.
  python tools/sq_summary.py gpurun_out/pmc_sq/run_counter_collection.csv <tag>
The pass covers the whole bench.py run (timing-mode eager steps included)."""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    tag = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    print("# SQ counters %s\n" % tag)
    print("One `rocprofv3 --pmc` pass over `bench.py --steps 5 --warmup 2 --no-cpu` (all dispatches, "
          "eager timing steps included). WAIT_ANY and ACTIVE_INST_ANY are fractions of "
          "SQ_WAVE_CYCLES (wave-cycles); VALU and VMEM_RD are instructions per wave.\n")
    print("| kernel | dispatches | waves | wait_any | active_inst | VALU/wave | VMEM_RD/wave | VALU per VMEM_RD |")
    print("|---|---|---|---|---|---|---|---|")
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0.0)):
        w = c.get("SQ_WAVES", 0.0)
        cyc = c.get("SQ_WAVE_CYCLES", 0.0)
        if w <= 0 or cyc <= 0:
            continue
        valu, vm = c.get("SQ_INSTS_VALU", 0.0), c.get("SQ_INSTS_VMEM_RD", 0.0)
        print("| `%s` | %d | %.0f | %.2f | %.2f | %.0f | %.1f | %s |" % (
            k, len(disp[k]), w, c.get("SQ_WAIT_ANY", 0.0) / cyc, c.get("SQ_ACTIVE_INST_ANY", 0.0) / cyc,
            valu / w, vm / w, ("%.0f" % (valu / vm)) if vm else "-"))


if __name__ == "__main__":
    main()
