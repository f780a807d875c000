# Round-end check on the final tree: full GPU suite, smoke and the default
# bench (its line, full object and the rocprofv3 stats CSVs it is priced on
# land in gpurun_out/$FINAL_TAG/; copy them to profiles/rNN/final/).
set -o pipefail
T=${FINAL_TAG:-final}
bash tools/gpu_session.sh $T tests smoke bench=--steps,20,--warmup,5
