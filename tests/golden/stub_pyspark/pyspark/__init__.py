"""Minimal, sequential, single-partition stand-in for the PySpark RDD API.

TEST INFRASTRUCTURE ONLY. Used exclusively by ``tests/golden/make_golden.py`` in the
build container to execute the reference's own ``coloring.py`` /
``coloring_optimized.py`` (which import pyspark at module top) so that golden
vectors can be recorded.  It never ships and never runs on the GPU box.

Ordering semantics modelled: the reference runs with
``spark.default.parallelism=1`` (coloring.py:196), i.e. one partition, so
* ``reduce`` is a left fold in RDD order,
* ``groupByKey`` lists values in RDD order, keys in first-seen order,
* ``aggregateByKey`` folds values in arrival (RDD) order from a deep copy of zero,
* ``leftOuterJoin`` keeps the left side's order.
"""
import copy
import functools


class StorageLevel:
    MEMORY_AND_DISK = "MEMORY_AND_DISK"


class Broadcast:
    def __init__(self, value):
        self.value = value


class RDD:
    def __init__(self, items):
        self._d = list(items)

    # narrow transformations
    def map(self, f):
        return RDD([f(x) for x in self._d])

    def filter(self, f):
        return RDD([x for x in self._d if f(x)])

    def flatMap(self, f):
        return RDD([y for x in self._d for y in f(x)])

    def mapValues(self, f):
        return RDD([(k, f(v)) for k, v in self._d])

    # actions
    def count(self):
        return len(self._d)

    def collect(self):
        return list(self._d)

    def collectAsMap(self):
        return dict(self._d)

    def reduce(self, f):
        if not self._d:
            raise ValueError("Can not reduce() empty RDD")
        return functools.reduce(f, self._d)

    def max(self):
        return max(self._d)

    def mean(self):
        return sum(self._d) / len(self._d)

    # partitioning / caching (single partition: identity)
    def getNumPartitions(self):
        return 1

    def partitionBy(self, n, partitionFunc=None):
        return RDD(self._d)

    def persist(self, level=None):
        return self

    def unpersist(self):
        return self

    # shuffles
    def groupByKey(self):
        groups = {}
        for k, v in self._d:
            groups.setdefault(k, []).append(v)
        return RDD(list(groups.items()))

    def aggregateByKey(self, zero, seq_func, comb_func):
        acc = {}
        for k, v in self._d:
            acc[k] = seq_func(acc[k] if k in acc else copy.deepcopy(zero), v)
        return RDD(list(acc.items()))

    def leftOuterJoin(self, other):
        right = {}
        for k, v in other._d:
            right.setdefault(k, []).append(v)
        return RDD([(k, (v, w)) for k, v in self._d for w in right.get(k, [None])])


class SparkContext:
    def parallelize(self, data):
        return RDD(data)

    def broadcast(self, value):
        return Broadcast(value)
