set -o pipefail
# timing-only ablations of the C2 schedule (layout 203, 2 groups; results WRONG by design): which
# wave's work sets the decision time (1 range-and-bearing, 2 proximity, 3 both, 4 robot pushes, 16 solver)
OUT=gpurun_out/r06s17 REPS=2 KS="2" LAYOUTS="0" VLIBS="product build/variants/lib_ab1.so build/variants/lib_ab2.so build/variants/lib_ab3.so build/variants/lib_ab4.so build/variants/lib_ab16.so" bash tools/groups_sweep.sh || exit 4
