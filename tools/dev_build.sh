#!/bin/bash
# Dev library with the ablation kernels (MP2VG_ABLATE) compiled in: tiny_mp2v_dec_amd/_var/dev/.
# The product library refuses MP2VG_ABLATE.  Use it as MP2VG_LIB=tiny_mp2v_dec_amd/_var/dev/libmp2vg.so
# with tools/stamps.py, abl_fused.sh, abl_sweep.sh, ablate.sh, c5_ablate.sh, profile_abl_counts.sh.
set -e
EXTRA=-DMP2VG_DEV_ABLATIONS tools/variant.sh dev tiny_mp2v_dec_amd/csrc/recon.hip
rm -f tiny_mp2v_dec_amd/_var/dev/*.o
