set -u
bash tools/ab_alt.sh r04_nt_c3 3 c3 base ntl nts ntls && bash tools/ab_alt.sh r04_nt_c4 2 c4 base ntls
