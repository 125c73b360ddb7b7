# ResNet-50 bench bs1024: shipped find DB vs copies preferring the CK backward-data solution
# (no fp32 workspace / zero-fill / cast passes) when within 10% / 30% of the ASM one
set -o pipefail
mkdir -p gpurun_out/ck_ab
python tools/miopen_prefer_ck.py tools/miopen/db /tmp/db_ck10 --dirs B --slack 1.10 > gpurun_out/ck_ab/gen.txt && \
python tools/miopen_prefer_ck.py tools/miopen/db /tmp/db_ck30 --dirs B --slack 1.30 >> gpurun_out/ck_ab/gen.txt && \
python tools/miopen_prefer_ck.py tools/miopen/db /tmp/db_ck30f --dirs F,B --slack 1.30 >> gpurun_out/ck_ab/gen.txt || exit 1
timeout -k 10 200 python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/ck_ab/import.txt 2>&1 || exit 1
for v in base ck10 ck30 ck30f base ck10 ck30 ck30f; do
  if [ $v = base ]; then db=$PWD/tools/miopen/db; else db=/tmp/db_$v; fi
  MIOPEN_USER_DB_PATH=$db timeout -k 10 200 python bench.py --steps 30 --warmup 8 > gpurun_out/ck_ab/$v.$RANDOM.txt 2>&1 || exit 1
done
