mkdir -p gpurun_out/exo3 && export TMPDIR=/tmp
for c in C3 C2 C4 C1; do
  O=orig,sort_src8,sort_src10,sort_src12
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/exo3/kt_$c -o kt --output-format csv -- python3 tools/exp_order.py --config $c --orders $O > gpurun_out/exo3/order_$c.jsonl 2> gpurun_out/exo3/order_$c.err || exit $?
  echo "== $c"; cat gpurun_out/exo3/order_$c.jsonl; python3 tools/kt_order.py gpurun_out/exo3/kt_$c/kt_kernel_trace.csv $O
done
