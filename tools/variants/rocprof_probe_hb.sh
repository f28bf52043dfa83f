export TMPDIR=/tmp
LIB=4dgaussians-fast-train_amd/diff_gaussian_rasterization/libgs4d.so
cp $LIB /tmp/libgs4d_intree.so
for v in hbcur hbnocomp; do
  cp variants/$v/libgs4d.so $LIB
  rm -rf gpurun_out/v_$v
  cd tools/probes && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ../../gpurun_out/v_$v -o run --output-format csv -- python3 heads_bwd_probe.py > ../../gpurun_out/v_$v.log 2>&1; cd ../..
done
cp /tmp/libgs4d_intree.so $LIB
