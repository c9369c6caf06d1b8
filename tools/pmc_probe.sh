set -u
cd $GRAFT_REPO_ROOT
for x in "" "-DFFD_TRAV_PROBE=1" "-DFFD_TRAV_PROBE=2"; do
  tag=$(echo "m$x" | tr -cd 'a-zA-Z0-9')
  rm -f face_alignment_cvpr_2012_amd/lib/*.o face_alignment_cvpr_2012_amd/lib/libffd.so
  make -j16 EXTRA="$x" face_alignment_cvpr_2012_amd/lib/libffd.so > /dev/null 2>&1 || exit 3
  PMC_GROUPS=$GRAFT_REPO_ROOT/tools/pmc_groups_mem.txt bash tools/pmc.sh $tag || exit $?
done
