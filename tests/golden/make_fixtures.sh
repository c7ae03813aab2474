#!/bin/sh
# Re-create the golden fixtures from a reference checkout (data files only).
set -e
R=${1:-/root/reference}/triplet_data
D=$(dirname "$0")
cp "$R/Figure_1/raw_data_8000.csv" "$D/fig1_raw_data_8000.csv"
cp "$R/Figure_1/astar_dag_8000.csv" "$D/fig1_astar_dag_8000.csv"
cp "$R/Figure_1/triplet_mec_8000.csv" "$D/fig1_triplet_mec_8000.csv"
cp "$R/Figure_2/raw_data_5000.csv" "$D/fig2_raw_data_5000.csv"
cp "$R/Figure_2/astar_dag_5000.csv" "$D/fig2_astar_dag_5000.csv"
cp "$R/Figure_2/triplet_mec_5000.csv" "$D/fig2_triplet_mec_5000.csv"
chmod 644 "$D"/*.csv
# Figure 3 learned A* DAGs (n=20, N=10000, seeds 9200-9229) and the Figure 4
# edge counts they reproduce (calc_dag_score's "edges" column)
mkdir -p "$D/fig3"
for s in $(seq 9200 9229); do cp "$R/Figure_3/learned_result/astar2_N10000_$s.csv" "$D/fig3/"; done
cp "$R/Figure_4/edge_true_astar_ges_10k_group2_lambda1.csv" "$D/fig4_edge_true_astar_ges_10k_group2_lambda1.csv"
chmod 644 "$D"/*.csv "$D"/fig3/*.csv
# Config C1's data (BASELINE.json configs[0]): the reference's data/hepatitis.clean.csv
cp "${1:-/root/reference}/data/hepatitis.clean.csv" "$D/hepatitis.clean.csv"
chmod 644 "$D/hepatitis.clean.csv"
