"""Write profiles/<NAME>.md, <NAME>_bench.json, <NAME>_kernels.json, <NAME>_kernel_stats.csv and refresh
profiles/latest_kernels.json / latest_knn_pmc.json (+ latest_kernels.meta.json: the commit and the kernel
sources' hash the profile was taken on, which bench.py reports beside the traffic it reads) from a
tools/gpu_round6.sh run (or $GPU_SCRIPT) in gpurun_out/.

usage: python tools/profile_note.py NAME "title" "command / commit note"
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def main():
    name, title, note = sys.argv[1:4]
    need = [os.path.join(G, "prof_kt", "kt_kernel_stats.csv"), os.path.join(G, "prof_fetch"), os.path.join(G, "prof_write"),
            os.path.join(G, "bench.json"), os.path.join(G, "gputest.log")]
    missing = [p for p in need if not os.path.exists(p)]
    if missing:  # a failed or partial session: change nothing under profiles/
        sys.exit(f"profile_note: missing {missing}")
    kj = os.path.join(P, f"{name}_kernels.json")
    table = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof_summary.py"), os.path.join(G, "prof_kt"),
                            os.path.join(G, "prof_fetch"), os.path.join(G, "prof_write")], check=True, capture_output=True,
                           text=True, env=dict(os.environ, PROF_JSON=kj)).stdout
    shutil.copy(kj, os.path.join(P, "latest_kernels.json"))
    sys.path.insert(0, ROOT)
    import bench
    # PROFILE_COMMIT: the commit the session ran on, when HEAD has moved on since (tests or docs only)
    head = os.environ.get("PROFILE_COMMIT") or subprocess.run(["git", "rev-parse", "HEAD"], cwd=ROOT,
                                                              capture_output=True, text=True).stdout.strip()
    dirty = subprocess.run(["git", "status", "--porcelain", "hidegs_amd/csrc", "include"], cwd=ROOT,
                           capture_output=True, text=True).stdout.strip() != ""
    box_sha = os.path.join(G, "sources.sha256")  # written on the GPU box by the session script
    sha = open(box_sha).read().strip() if os.path.exists(box_sha) else bench.sources_sha256()
    with open(os.path.join(P, "latest_kernels.meta.json"), "w") as f:
        json.dump({"commit": head[:12] + ("+uncommitted kernel edits" if dirty else ""), "sources_sha256": sha,
                   "profile": name, "command": "tools/gpu_round5.sh / gpu_round6.sh: rocprofv3 --kernel-trace --stats, then "
                   "--pmc FETCH_SIZE and --pmc WRITE_SIZE passes of bench.py", "note": note}, f, indent=1)
    shutil.copy(os.path.join(G, "prof_kt", "kt_kernel_stats.csv"), os.path.join(P, f"{name}_kernel_stats.csv"))
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_json.py"), os.path.join(G, "prof_knn"),
                    os.path.join(P, "latest_knn_pmc.json"), "knn_leaf"], check=True, capture_output=True)
    line = open(os.path.join(G, "bench.json")).read().strip().splitlines()[-1]
    with open(os.path.join(P, f"{name}_bench.json"), "w") as f:
        f.write(line + "\n")
    d = json.loads(line)
    b, r = d["binning_step"], d["roofline"]
    tests = open(os.path.join(G, "gputest.log")).read().strip().splitlines()[-1]
    with open(os.path.join(P, f"{name}.md"), "w") as f:
        f.write(f"# {title}\n\n")
        f.write(f"Command: `{os.environ.get('GPU_SCRIPT', 'tools/gpu_round6.sh')}` ({note}; tests: {tests}; smoke; bench; rocprofv3 kernel trace; "
                "FETCH_SIZE / WRITE_SIZE passes; knn VALU pass).\n")
        f.write(f"Bench line: `{name}_bench.json`: binning step {b['ms_per_step']} ms (radix_scatter {r['avg_launch_us']} us "
                f"in-bench = {r['frac']} of 8 TB/s; traffic {r['traffic'] / 1e6:.1f} MB against "
                f"{r['algorithmic_bytes_per_launch'] / 1e6:.1f} MB algorithmic), skewed view {d['binning_skewed']['ms_per_step']} ms, "
                f"distCUDA2 {d['distCUDA2']['ms']} ms (knn_leaf issue frac {d['distCUDA2']['issue_roofline']['frac']}), "
                f"masked Adam {d['masked_adam']['ms']} ms, dp_step {d['dp_step']['fp32_ms_per_step']} / "
                f"{d['dp_step']['bf16_ms_per_step']} ms (fp32 / bf16 wire), forced one-rank exchange "
                f"{d['exchange']['forced_one_rank_rccl']['ms_per_step']} / {d['exchange_bf16']['forced_one_rank_rccl']['ms_per_step']} ms, "
                f"config 5 binning {d['config5_scale']['binning_ms_per_step']} ms / distCUDA2 {d['config5_scale']['distCUDA2_ms']} ms, "
                f"CPU baseline {d['cpu_baseline']['value'] / 1e6:.0f}M pairs/s ({d['cpu_baseline']['cores']} threads, "
                f"{d['cpu_baseline']['cpu']}).\n")
        f.write("Corrected HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB per launch (MI355X_MICROARCH.md).\n\n")
        f.write(table)


if __name__ == "__main__":
    main()
