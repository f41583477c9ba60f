#!/bin/bash
cd "$(dirname "$0")"
for b in lin2_pf*; do timeout -k 5 60 ./$b; done
