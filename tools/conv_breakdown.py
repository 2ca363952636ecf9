"""Per-launch breakdown of the po_conv kernel from a rocprofv3 kernel trace:
maps the conv_k dispatches of the last step onto the Darknet plan's launch
list and prints time, algorithmic TFLOP/s per launch, grouped by layer."""
import csv, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import __graft_entry__ as ge

trace, cfg, B = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = [r for r in csv.DictReader(open(trace)) if r["Kernel_Name"].startswith("conv_k")]
dk = ge._pkg("darknet_v3")
W = ge._pkg("weights")
net = dk.Darknet(cfg)
W.write_weights("/tmp/cb.weights", W.synthesize(cfg))
net.load_darknet_weights("/tmp/cb.weights")
S = net.height
plan = net.plan(B, S, S, torch.device("cpu"))
launches = []
for phase, ops in (("fwd", plan.fwd_ops), ("bwd", plan.bwd_ops)):
    for name, args, desc in ops:
        if name != "po_conv":
            continue
        M = desc.B * desc.Hg * desc.Wg
        K = desc.ntaps * desc.Cin_p
        launches.append((phase, M, desc.N, K, desc.ntaps, desc.Cin_p))
n = len(launches)
last = rows[-n:]
tot_t = 0; tot_f = 0
print("%-4s %8s %5s %6s %9s %8s %7s" % ("ph", "M", "N", "K", "us", "TFLOP/s", "grid"))
for (ph, M, N, K, nt, cin), r in zip(launches, last):
    t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    fl = 2.0 * M * N * K
    tot_t += t; tot_f += fl
    print("%-4s %8d %5d %6d %9.1f %8.1f %7s" % (ph, M, N, K, t, fl / t / 1e6, r["Grid_Size_X"]))
print("total conv us %.1f  padded-FLOP rate %.1f TFLOP/s" % (tot_t, tot_f / tot_t / 1e6))
