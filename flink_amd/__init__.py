"""flink_amd: MI355X-native windowed keyed-aggregation hot path of Apache Flink."""
__version__ = "0.1.0"
