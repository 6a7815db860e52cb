#!/bin/bash
# run-cpu.sh -- the reference's benchmark harness (scripts/run-cpu.sh:1-86 of GenomicsBench) over the
# MI355X drop-ins: same <INPUTS_DIR> layout, same per-benchmark command lines, with
# genomicsbench_palisade_amd/bin/{fmi,bsw,phmm,chain} in place of ../benchmarks/*/. The name is kept so
# existing invocations work unchanged; the four hot kernels run on the GPU ($GB_DEVICE, default 0).
#   scripts/run-cpu.sh <INPUTS_DIR> <small|large> [fmi bsw phmm chain ...]
# With no benchmark list all four run (phmm, commented out in the reference, is included). dbg, poa,
# kmer-cnt, pileup and grm are not part of this framework and are reported as
# skipped. scripts/make-inputs.py writes a synthetic <INPUTS_DIR> in this layout.
# Optional outputs (unset: the reference's command lines exactly): GB_BSW_OUT=<file> writes bsw's
# per-pair score/qle/tle/gtle/gscore/max_off lines; GB_PHMM_PRINT=1 prints every phmm result ("%lf").
set -e

usage() {
	echo -e "\n Usage $0 <INPUTS_DIR> <INPUT_SIZE> [benchmark ...]\n\n Example: $0 [../input-datasets] [small | large] [fmi bsw phmm chain]\n"
}

if [[ ( $1 == "--help" ) || ( $1 == "-h" ) ]]; then
	usage
	exit 0
fi
if [[ $# -lt 1 ]]; then
	usage
	exit 1
fi

HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
BIN="$HERE/../genomicsbench_palisade_amd/bin"
INPUTS_DIR=$1
INPUTS_SIZE=${2:-small}
shift $(( $# >= 2 ? 2 : 1 ))
BENCHES=${*:-"fmi bsw phmm chain dbg poa kmer-cnt pileup grm"}

if [[ $INPUTS_SIZE == "large" ]]; then
	FMI_READS=$INPUTS_DIR/fmi/large/SRR7733443_10m_1.fastq
	BSW_PAIRS=$INPUTS_DIR/bsw/large/bandedSWA_SRR7733443_1m_input.txt
	PHMM_IN=$INPUTS_DIR/phmm/large/large.in
	CHAIN_IN=$INPUTS_DIR/chain/large/c_elegans_40x.10k.in
	CHAIN_OUT=$INPUTS_DIR/chain/large/c_elegans_40x.10k.out
else
	FMI_READS=$INPUTS_DIR/fmi/small/SRR7733443_1m_1.fastq
	BSW_PAIRS=$INPUTS_DIR/bsw/small/bandedSWA_SRR7733443_100k_input.txt
	PHMM_IN=$INPUTS_DIR/phmm/small/5m.in
	CHAIN_IN=$INPUTS_DIR/chain/small/in-1k.txt
	CHAIN_OUT=$INPUTS_DIR/chain/small/out-1k.txt
fi

for b in $BENCHES; do
	case $b in
	fmi)
		echo "Running fmi"
		"$BIN/fmi" "$INPUTS_DIR/fmi/broad" "$FMI_READS" 512 19 1
		;;
	bsw)
		echo "Running bsw"
		"$BIN/bsw" -pairs "$BSW_PAIRS" -t 1 -b 512 ${GB_BSW_OUT:+-o "$GB_BSW_OUT"}
		;;
	phmm)
		echo "Running phmm"
		"$BIN/phmm" -f "$PHMM_IN" -t 1 ${GB_PHMM_PRINT:+-p}
		;;
	chain)
		echo "Running chain"
		"$BIN/chain" -i "$CHAIN_IN" -o "$CHAIN_OUT"
		;;
	dbg | poa | kmer-cnt | pileup | grm)
		echo "Skipping $b (not one of the MI355X hot kernels: fmi, bsw, phmm, chain)"
		;;
	*)
		echo "unknown benchmark: $b" >&2
		usage
		exit 1
		;;
	esac
done
