set -u
bash tools/ab_alt.sh r04_nt2_c4 2 c4 base ntl nts && bash tools/ab_alt.sh r04_nt2_c2 3 c2 base ntl nts ntls
