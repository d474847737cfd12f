"""Command-line entrypoints (hipKNN_unorderedData, hipKNN_prePartitionedData, tools)."""
