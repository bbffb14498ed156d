cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hashab
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
Q="--threads= --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0 --other-mix 0 --steps 30"
bash scripts/gpu_session.sh \
 "ab4k:200:CONFIGS='base:;p41:SDFS_HASH_VARIANT=41;p40:SDFS_HASH_VARIANT=40;p42:SDFS_HASH_VARIANT=42' ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "abdef:200:CONFIGS='base:;p41:SDFS_HASH_VARIANT=41;p40:SDFS_HASH_VARIANT=40' ROUNDS=8 python3 scripts/ab.py" \
 "b_base:120:python3 bench.py $Q" \
 "b_p41:120:SDFS_HASH_VARIANT=41 python3 bench.py $Q" \
 "b_base2:120:python3 bench.py $Q" \
 "b_p41b:120:SDFS_HASH_VARIANT=41 python3 bench.py $Q" \
 "inproc:120:unset SDFS_CDC_LIB; python3 bench.py --inproc 1 --steps 20"
