"""SparkSession stand-in for the golden-vector generator (test infrastructure only)."""
from pyspark import SparkContext


class _Builder:
    def appName(self, *args):
        return self

    def master(self, *args):
        return self

    def config(self, *args):
        return self

    def getOrCreate(self):
        return SparkSession()


class SparkSession:
    builder = _Builder()

    def __init__(self):
        self.sparkContext = SparkContext()

    def stop(self):
        pass
