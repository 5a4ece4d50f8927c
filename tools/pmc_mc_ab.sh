bash tools/pmc_mc.sh new && VVCR_LIB=vvc_amd/libvvcr_old.so bash tools/pmc_mc.sh old
