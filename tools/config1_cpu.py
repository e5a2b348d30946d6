#!/usr/bin/env python3
"""BASELINE config 1 on the host CPU: RAID5 4+1 full-stripe writes of 256 KiB
(64 KiB strips) over 5 RAM disks, bdevperf-style (oracle/bdevperf_raid5.c).
Writes gpurun_out/config1_cpu.json."""
import json
import os
import platform
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    secs = float(os.environ.get("SECONDS_RUN", "10"))
    qd = int(os.environ.get("QD", "32"))
    mibs, ios, ok = oracle.bdevperf_raid5_fsw(n=5, strip=65536, disk_bytes=1 << 30, seconds=secs,
                                              qd=qd)
    r = {"config": "RAID5 4+1 full-stripe write, 64 KiB strip, bdevperf-style over 5 RAM disks",
         "io_size": 262144, "qd": qd, "cores": 1, "seconds": secs, "ios": ios,
         "mib_s": round(mibs, 1),
         "iops": round(ios / secs, 1), "parity_verified": ok, "cpu": cpu_model(),
         "xor_gen": "AVX-512 restatement of isa-l xor_gen_avx512 (oracle/isal_simd.c)"
         if oracle.simd_available() else "scalar restatement",
         "kind": "port (oracle xor_gen restatement + memcpy per strip)"}
    print(json.dumps(r))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "config1_cpu.json"), "w") as f:
        json.dump(r, f, indent=1)


if __name__ == "__main__":
    main()
