bash tools/variants/sq_variants.sh base && bash tools/variants/run_variants.sh base tail4096 tail2720
