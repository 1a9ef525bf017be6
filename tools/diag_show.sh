#!/bin/bash
for v in ${VARIANTS:-full diag1 diag2 diag3 diag4}; do python3 -c "
import csv,sys
r=list(csv.reader(open('gpurun_out/diag_$v/run_kernel_stats.csv')))
for row in r[1:]:
  if 'fks' in row[0]: print('$v', row[0][30:62], row[1], round(float(row[3])/1e6,4),'ms')"; done
