#!/bin/bash
# A/B of two libqfec.so builds (tools/ab/old.so, tools/ab/new.so) on the
# service's per-call host cost (tools/tune/build/svc_host_cost), alternating.
cp libquic_amd/libqfec.so /tmp/orig_libqfec.so
for round in 1 2; do
  for v in ${ORDER:-old new}; do
    cp tools/ab/$v.so libquic_amd/libqfec.so
    for g in 5 20 200; do
      echo -n "$v $round "; timeout -k 10 60 tools/tune/build/svc_host_cost $g || { cp /tmp/orig_libqfec.so libquic_amd/libqfec.so; exit 1; }
    done
  done
done
cp /tmp/orig_libqfec.so libquic_amd/libqfec.so
