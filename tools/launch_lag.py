#!/usr/bin/env python3
"""Host launch time against GPU start of each kernel (diagnostics): joins a
rocprofv3 kernel trace with its HIP API trace by correlation id and prints, for
the last kernels, when the host called the launch, when the kernel began and
ended (us, relative), and the lag between the call and the start.

    python tools/launch_lag.py gpurun_out/r5p [--last 40]
"""
import argparse
import csv
import glob
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=40)
    a = ap.parse_args()
    kt = glob.glob(a.dir + "/**/*kernel_trace.csv", recursive=True)[0]
    ht = glob.glob(a.dir + "/**/*hip_api_trace.csv", recursive=True)[0]
    api = {}
    for r in csv.DictReader(open(ht)):
        api[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                    r["Function"])
    ks = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))[-a.last:]
    t0 = min(min(int(r["Start_Timestamp"]) for r in ks),
             min(api[r["Correlation_Id"]][0] for r in ks if r["Correlation_Id"] in api))
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("misor::", "")
        c = api.get(r["Correlation_Id"])
        call = (c[0] - t0) / 1e3 if c else float("nan")
        print("call %9.1f  start %9.1f  end %9.1f  lag %8.1f  q%-3s %s" % (
            call, (s - t0) / 1e3, (e - t0) / 1e3, (s - c[0]) / 1e3 if c else float("nan"),
            r.get("Queue_Id", ""), name[:50]))


if __name__ == "__main__":
    main()
