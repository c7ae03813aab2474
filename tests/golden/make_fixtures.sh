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
