"""Write reference_kats.json: the reference's own hot-path fixtures and known answers.

Every dataset is transcribed from the reference's test fixtures and every expected value
from an assertion in the reference's test suite (paths relative to
src/test/scala/com/amazon/deequ/).  This is data only: tables + expected metrics.
`expected` is a float, "NaN", "EmptyState" (metric fails with EmptyStateException,
Analyzer.scala:420-431), or {"DataTypeHistogram": [numNull, numFractional, numIntegral,
numBoolean, numString]} for DataType (its HistogramMetric is DataTypeHistogram.toDistribution of
that state, DataType.scala:98-114).  `needs` lists GPU-path capabilities a case depends on that the GPU path does not
have (e.g. a regex outside the GPU subset), so tests expect the fallback route for it.
"""
import json
import math
import os

N = None

datasets = {
    "dfMissing": {  # utils/FixtureSupport.scala:45-62
        "columns": {
            "item": ["utf8", [str(i) for i in range(1, 13)]],
            "att1": ["utf8", ["a", "b", N, "a", "a", N, N, "b", "a", N, N, N]],
            "att2": ["utf8", ["f", "d", "f", N, "f", "d", "d", N, "f", N, "f", "d"]],
        }
    },
    "dfFull": {  # utils/FixtureSupport.scala:64-73
        "columns": {
            "item": ["utf8", ["1", "2", "3", "4"]],
            "att1": ["utf8", ["a", "a", "a", "b"]],
            "att2": ["utf8", ["c", "c", "c", "d"]],
        }
    },
    "dfWithNumericValues": {  # utils/FixtureSupport.scala:137-148 (att1, att2: Int)
        "columns": {
            "item": ["utf8", ["1", "2", "3", "4", "5", "6"]],
            "att1": ["i32", [1, 2, 3, 4, 5, 6]],
            "att2": ["i32", [0, 0, 0, 5, 6, 7]],
        }
    },
    "dfWithNumericFractionalValues": {  # utils/FixtureSupport.scala:150-160
        "columns": {
            "item": ["utf8", ["1", "2", "3", "4", "5", "6"]],
            "att1": ["f64", [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]],
            "att2": ["f64", [0.0, 0.0, 0.0, 5.0, 6.0, 7.0]],
        }
    },
    "dfWithNegativeNumbers": {  # utils/FixtureSupport.scala:75-84
        "columns": {
            "item": ["utf8", ["1", "2", "3", "4"]],
            "att1": ["utf8", ["-1", "-2", "-3", "-4"]],
            "att2": ["utf8", ["-1.0", "-2.0", "-3.0", "-4.0"]],
        }
    },
    "dfFractionalIntegralTypes": {  # utils/FixtureSupport.scala:110-117
        "columns": {"item": ["utf8", ["1", "2"]], "att1": ["utf8", ["1.0", "1"]]}
    },
    "dfFractionalStringTypes": {  # utils/FixtureSupport.scala:119-126
        "columns": {"item": ["utf8", ["1", "2"]], "att1": ["utf8", ["1.0", "a"]]}
    },
    "dfIntegralStringTypes": {  # utils/FixtureSupport.scala:128-135
        "columns": {"item": ["utf8", ["1", "2"]], "att1": ["utf8", ["1", "a"]]}
    },
    "dfWithNumericValuesAsString": {  # AnalyzerTests.scala:331-332: getDfWithNumericValues, att1 cast to string
        "columns": {"item": ["utf8", ["1", "2", "3", "4", "5", "6"]],
                    "att1_str": ["utf8", ["1", "2", "3", "4", "5", "6"]]}
    },
    "dfWithNumericFractionalValuesAsString": {  # AnalyzerTests.scala:338-339: Double att1 cast to string
        "columns": {"item": ["utf8", ["1", "2", "3", "4", "5", "6"]],
                    "att1_str": ["utf8", ["1.0", "2.0", "3.0", "4.0", "5.0", "6.0"]]}
    },
    "dfBoolean": {  # AnalyzerTests.scala:395-398
        "columns": {"item": ["utf8", ["1", "2"]], "att1": ["utf8", ["true", "false"]]}
    },
    "dfBooleanNullFractional": {  # AnalyzerTests.scala:407-412
        "columns": {"item": ["utf8", ["1", "2", "3", "4"]], "att1": ["utf8", ["true", "false", N, "2.0"]]}
    },
    "dfWithUniqueColumns": {  # utils/FixtureSupport.scala:162-175
        "columns": {
            "unique": ["utf8", ["1", "2", "3", "4", "5", "6"]],
            "nonUnique": ["utf8", ["0", "0", "0", "5", "6", "7"]],
            "nonUniqueWithNulls": ["utf8", ["3", "3", "3", N, N, N]],
            "uniqueWithNulls": ["utf8", ["1", "2", N, "3", "4", "5"]],
            "onlyUniqueWithOtherNonUnique": ["utf8", ["5", "6", "7", "0", "0", "0"]],
            "halfUniqueCombinedWithNonUnique": ["utf8", ["0", "0", "0", "4", "5", "6"]],
        }
    },
    "dfWithConditionallyUninformativeColumns": {  # utils/FixtureSupport.scala:190-197
        "columns": {"att1": ["i32", [1, 2, 3]], "att2": ["i32", [0, 0, 0]]}
    },
    "dfWithConditionallyInformativeColumns": {  # utils/FixtureSupport.scala:199-206
        "columns": {"att1": ["i32", [1, 2, 3]], "att2": ["i32", [4, 5, 6]]}
    },
    "dataWithNullColumns": {  # analyzers/NullHandlingTests.scala:32-50 (numSlices = 2)
        "partitions": 2,
        "columns": {
            "stringCol": ["utf8", [N] * 8],
            "numericCol": ["f64", [N] * 8],
            "numericCol2": ["f64", [N] * 8],
            "numericCol3": ["f64", [1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0]],
        },
    },
    "incrementalInitial": {  # analyzers/IncrementalAnalyzerTest.scala (initialData)
        "columns": {
            "item": ["utf8", ["1", "2", "3"]],
            "att1": ["utf8", ["a", "b", N]],
        }
    },
    "stateAggregation": {  # analyzers/StateAggregationIntegrationTest.scala:34-50
        "partitions": 2,
        "columns": {
            "item": ["utf8", ["item1", "item1", "item1", "item2", "item2", "item3", "item4", "item5"]],
            "origin": ["utf8", ["US", "US", "US", "DE", "DE", N, N, N]],
            "sales": ["i32", [100, 1000, 20, 20, 333, 12, 45, 123]],
            "marketplace": ["utf8", ["EU", "NA", "IN", "EU", "NA", "NA", "NA", "NA"]],
        },
    },
    # PatternMatch (AnalyzerTests.scala:626-721, checks/CheckTest.scala:352-476)
    "patternDoubles": {  # AnalyzerTests.scala:628-630 (DoubleType column: Spark casts it to string)
        "columns": {"some": ["f64", [1.1, N, 3.2, 4.4]]}
    },
    "patternIntegers": {"columns": {"some": ["utf8", ["1", "a"]]}},  # :635
    "patternEmails": {"columns": {"some": ["utf8", ["someone@somewhere.org", "someone@else"]]}},  # :641-642
    "patternCreditCards": {"columns": {"some": ["utf8", [  # :648-664
        "378282246310005", "6011111111111117", "6011 1111 1111 1117", "6011-1111-1111-1117",
        "5555555555554444", "5555 5555 5555 4444", "5555-5555-5555-4444", "4111111111111111",
        "4111 1111 1111 1111", "4111-1111-1111-1111", "0000111122223333", "000011112222333", "00001111222233"]]}},
    "patternUrls": {"columns": {"some": ["utf8", [  # :674-693 (incl. non-ASCII hosts / paths)
        "http://foo.com/blah_blah", "http://foo.com/blah_blah_(wikipedia)",
        "http://foo.bar/?q=Test%20URL-encoded%20stuff", "http://\u27a1.ws/\u4a39", "http://\u2318.ws/",
        "http://\u263a.damowmow.com/", "http://\u4f8b\u5b50.\u6d4b\u8bd5", "https://foo_bar.example.com/",
        "http://userid@example.com:8080", "http://foo.com/blah_(wikipedia)#cite-1", "http://../", "h://test",
        "http://.www.foo.bar/"]]}},
    "patternSsns": {"columns": {"some": ["utf8", [  # :703-712
        "111-05-1130", "111051130", "111-05-000", "111-00-000", "000-05-1130", "666-05-1130", "900-05-1130",
        "999-05-1130"]]}},
    "checkUrls": {"columns": {"some": ["utf8", [  # checks/CheckTest.scala:383-386
        "https://www.example.com/foo/?bar=baz&inga=42&quux", "http:// shouldfail.com"]]}},
    "checkEmails": {"columns": {"some": ["utf8", ["someone@somewhere.org", "someone@else.com"]]}},  # :354-355
    # checks/CheckTest.scala:765-785 (runAndAssertSuccessFor): one column "some" of each numeric type, rows
    # (1, null) -- isNonNegative / isPositive for ByteType .. DoubleType (:478-489)
    **{f"numericRowNull_{t}": {"columns": {"some": [t, [1.0 if t.startswith("f") else 1, N]]}}
       for t in ("i8", "i16", "i32", "i64", "f32", "f64")},
    # AnalyzerTests.scala:322-328: getDfWithNumericValues with att1 cast to FloatType
    "dfWithNumericValuesAsFloat": {
        "columns": {"item": ["utf8", ["1", "2", "3", "4", "5", "6"]],
                    "att1_float": ["f32", [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]]}
    },
    # profiles/ColumnProfilerTest.scala:177-190: a BooleanType column (true x3, false x2, null)
    "dfBooleanColumn": {"columns": {"attribute": ["bool", [True, True, True, False, False, N]]}},
    # AnalyzerTests.scala:489-505: a DecimalType.SYSTEM_DEFAULT = DecimalType(38, 18) column (values as decimal text)
    "dfDecimalSystemDefault": {"columns": {"num": ["decimal(38,18)", ["123.45", "99", "678"]]}},
    # constraints/ConstraintsTest.scala:126-146: dataFrameWithColumn(column, DoubleType / StringType, Row(..), Row(..))
    "dfDoubleColumn": {"columns": {"column": ["f64", [1.0, 2.0]]}},
    "dfStringNumericColumn": {"columns": {"column": ["utf8", ["1", "2.0"]]}},
}

S = "analyzers/AnalyzerTests.scala"
EMAIL = (r"""(?:[a-z0-9!#$%&'*+/=?^_`{|}~-]+(?:\.[a-z0-9!#$%&'*+/=?^_`{|}~-]+)*|"(?:[\x01-\x08\x0b\x0c\x0e-\x1f\x21\x23-\x5b\x5d-\x7f]|\\[\x01-\x09\x0b\x0c\x0e-\x7f])*")"""
         r"""@(?:(?:[a-z0-9](?:[a-z0-9-]*[a-z0-9])?\.)+[a-z0-9](?:[a-z0-9-]*[a-z0-9])?|\[(?:(?:25[0-5]|2[0-4][0-9]|[01]?[0-9][0-9]?)\.){3}"""
         r"""(?:25[0-5]|2[0-4][0-9]|[01]?[0-9][0-9]?|[a-z0-9-]*[a-z0-9]:(?:[\x01-\x08\x0b\x0c\x0e-\x1f\x21-\x5a\x53-\x7f]|\\[\x01-\x09\x0b\x0c\x0e-\x7f])+)\])""")
URL = r"""(https?|ftp)://[^\s/$.?#].[^\s]*"""
SSN = (r"""((?!219-09-9999|078-05-1120)(?!666|000|9\d{2})\d{3}-(?!00)\d{2}-(?!0{4})\d{4})|"""
       r"""((?!219 09 9999|078 05 1120)(?!666|000|9\d{2})\d{3} (?!00)\d{2} (?!0{4})\d{4})|"""
       r"""((?!219099999|078051120)(?!666|000|9\d{2})\d{3}(?!00)\d{2}(?!0{4})\d{4})""")
CREDITCARD = r"""\b(?:3[47]\d{2}([\ \-]?)\d{6}\1\d|(?:(?:4\d|5[1-5]|65)\d{2}|6011)([\ \-]?)\d{4}\2\d{4}\2)\d{4}\b"""
cases = [
    # Size / Completeness
    ("dfMissing", ["Size", N], 12.0, S + ":39-42", []),
    ("dfFull", ["Size", N], 4.0, S + ":39-42", []),
    ("dfMissing", ["Completeness", "att1", N], 0.5, S + ":52-53", []),
    ("dfMissing", ["Completeness", "att2", N], 0.75, S + ":54-55", []),
    ("dfMissing", ["Completeness", "att1", "item IN ('1', '2')"], 1.0, S + ":73-74", []),
    # Compliance
    ("dfWithNumericValues", ["Compliance", "rule1", "att1 > 3", N], 3.0 / 6, S + ":175-176", []),
    ("dfWithNumericValues", ["Compliance", "rule2", "att1 > 2", N], 4.0 / 6, S + ":177-178", []),
    ("dfWithNumericValues", ["Compliance", "rule1", "att2 = 0", "att1 < 4"], 1.0, S + ":184-185", []),
    # basic statistics
    ("dfWithNumericValues", ["Mean", "att1", N], 3.5, S + ":427-428", []),
    ("dfWithNumericValues", ["Mean", "att1", "item != '6'"], 3.0, S + ":437-438", []),
    ("dfWithNumericValues", ["StandardDeviation", "att1", N], 1.707825127659933, S + ":443-444", []),
    ("dfWithNumericValues", ["Minimum", "att1", N], 1.0, S + ":453-454", []),
    ("dfWithNumericValues", ["Maximum", "att1", N], 6.0, S + ":463-464", []),
    ("dfWithNumericValues", ["Maximum", "att1", "item != '6'"], 5.0, S + ":470-471", []),
    ("dfWithNumericValues", ["Sum", "att1", N], 21.0, S + ":481", []),
    # HLL
    ("dfWithUniqueColumns", ["ApproxCountDistinct", "uniqueWithNulls", N], 5.0, S + ":509-513", []),
    # Correlation
    ("dfWithConditionallyUninformativeColumns", ["Correlation", "att1", "att2", N], "NaN", S + ":604-608", []),
    ("dfWithConditionallyInformativeColumns", ["Correlation", "att1", "att2", N], 1.0, S + ":610-617", []),
    ("dfWithConditionallyInformativeColumns", ["Correlation", "att2", "att1", N], 1.0, S + ":619-623", []),
    # fused runner (analyzers/AnalysisTest.scala:86-92)
    ("dfWithNumericValues", ["ApproxCountDistinct", "att1", N], 6.0, "analyzers/AnalysisTest.scala:91-92", []),
    # null handling (analyzers/NullHandlingTests.scala:87-118)
    ("dataWithNullColumns", ["Size", N], 8.0, "analyzers/NullHandlingTests.scala:91", []),
    ("dataWithNullColumns", ["Completeness", "stringCol", N], 0.0, "analyzers/NullHandlingTests.scala:92", []),
    ("dataWithNullColumns", ["Mean", "numericCol", N], "EmptyState", "analyzers/NullHandlingTests.scala:94", []),
    ("dataWithNullColumns", ["StandardDeviation", "numericCol", N], "EmptyState", "analyzers/NullHandlingTests.scala:96", []),
    ("dataWithNullColumns", ["Minimum", "numericCol", N], "EmptyState", "analyzers/NullHandlingTests.scala:97", []),
    ("dataWithNullColumns", ["Maximum", "numericCol", N], "EmptyState", "analyzers/NullHandlingTests.scala:98", []),
    ("dataWithNullColumns", ["Sum", "numericCol", N], "EmptyState", "analyzers/NullHandlingTests.scala:103", []),
    ("dataWithNullColumns", ["ApproxCountDistinct", "stringCol", N], 0.0, "analyzers/NullHandlingTests.scala:107", []),
    ("dataWithNullColumns", ["Correlation", "numericCol", "numericCol2", N], "EmptyState", "analyzers/NullHandlingTests.scala:114", []),
    ("dataWithNullColumns", ["Correlation", "numericCol", "numericCol3", N], "EmptyState", "analyzers/NullHandlingTests.scala:115", []),
    # checks -> Compliance (checks/CheckTest.scala:156-273), metric values implied by the statuses
    ("dfWithNumericValues", ["Compliance", "rule1", "att1 > 0", N], 1.0, "checks/CheckTest.scala:158-170", []),
    ("dfWithNumericValues", ["Compliance", "rule1", "att1 < att2", "att1 > 3"], 1.0, "checks/CheckTest.scala:176-192", []),
    ("dfWithNumericValues", ["Compliance", "rule2", "att2 > 0", "att1 > 0"], 0.5, "checks/CheckTest.scala:179-192", []),
    ("dfWithNumericValues", ["Compliance", "att1 is less than att2", "att1 < att2", N], 0.5, "checks/CheckTest.scala:200-213", []),
    ("dfWithNumericValues", ["Compliance", "nr1", "`att2` IS NULL OR (`att2` >= 0.0 AND `att2` <= 7.0)", N], 1.0, "checks/CheckTest.scala:235-267; Check.scala:867-868", []),
    ("dfWithNumericValues", ["Compliance", "nr2", "`att2` IS NULL OR (`att2` >= 1.0 AND `att2` <= 7.0)", N], 0.5, "checks/CheckTest.scala:238-268", []),
    ("dfWithNumericValues", ["Compliance", "nr3", "`att2` IS NULL OR (`att2` >= 0.0 AND `att2` <= 6.0)", N], 5.0 / 6, "checks/CheckTest.scala:241-269", []),
    ("dfWithNumericValues", ["Compliance", "nr4", "`att2` IS NULL OR (`att2` > 0.0 AND `att2` < 7.0)", N], 2.0 / 6, "checks/CheckTest.scala:244-270", []),
    ("dfWithNumericValues", ["Compliance", "nr5", "`att2` IS NULL OR (`att2` > -1.0 AND `att2` < 8.0)", N], 1.0, "checks/CheckTest.scala:247-271", []),
    ("dfWithNumericValues", ["Compliance", "nr6", "`att2` IS NULL OR (`att2` >= 0.0 AND `att2` < 7.0)", N], 5.0 / 6, "checks/CheckTest.scala:250-272", []),
    ("dfWithNumericValues", ["Compliance", "nr7", "`att2` IS NULL OR (`att2` >= 0.0 AND `att2` < 8.0)", N], 1.0, "checks/CheckTest.scala:253-273", []),
    ("dfWithNumericValues", ["Compliance", "nr8", "`att2` IS NULL OR (`att2` > 0.0 AND `att2` <= 7.0)", N], 3.0 / 6, "checks/CheckTest.scala:256-274", []),
    ("dfWithNumericValues", ["Compliance", "nr9", "`att2` IS NULL OR (`att2` > -1.0 AND `att2` <= 7.0)", N], 1.0, "checks/CheckTest.scala:259-275", []),
    ("dfWithNumericValues", ["Compliance", "att1 is non-negative", "COALESCE(att1, 0.0) >= 0", N], 1.0, "predicate form Check.scala:676 (isNonNegative); expected value computed by hand", []),
    ("dfWithNumericValues", ["Compliance", "att2 is positive", "COALESCE(att2, 1.0) > 0", N], 0.5, "predicate form Check.scala:687 (isPositive); expected value computed by hand", []),
    # DataType (AnalyzerTests.scala:295-421; the FloatType case :322-328 is below with the round-6 column types)
    ("dfFull", ["DataType", "att1", N], {"DataTypeHistogram": [0, 0, 0, 0, 4]}, S + ":295-300", []),
    ("dfWithNumericValues", ["DataType", "att1", N], {"DataTypeHistogram": [0, 0, 6, 0, 0]}, S + ":302-306", []),
    ("dfWithNegativeNumbers", ["DataType", "att1", N], {"DataTypeHistogram": [0, 0, 4, 0, 0]}, S + ":308-312", []),
    ("dfWithNegativeNumbers", ["DataType", "att2", N], {"DataTypeHistogram": [0, 4, 0, 0, 0]}, S + ":314-319", []),
    ("dfWithNumericValuesAsString", ["DataType", "att1_str", N], {"DataTypeHistogram": [0, 0, 6, 0, 0]}, S + ":330-335", []),
    ("dfWithNumericFractionalValuesAsString", ["DataType", "att1_str", N], {"DataTypeHistogram": [0, 6, 0, 0, 0]}, S + ":337-344", []),
    ("dfFractionalIntegralTypes", ["DataType", "att1", N], {"DataTypeHistogram": [0, 1, 1, 0, 0]}, S + ":353-361", []),
    ("dfFractionalStringTypes", ["DataType", "att1", N], {"DataTypeHistogram": [0, 1, 0, 0, 1]}, S + ":363-371", []),
    ("dfIntegralStringTypes", ["DataType", "att1", N], {"DataTypeHistogram": [0, 0, 1, 0, 1]}, S + ":373-381", []),
    ("dfWithUniqueColumns", ["DataType", "uniqueWithNulls", N], {"DataTypeHistogram": [1, 0, 5, 0, 0]}, S + ":383-391", []),
    ("dfBoolean", ["DataType", "att1", N], {"DataTypeHistogram": [0, 0, 0, 2, 0]}, S + ":393-403", []),
    ("dfBooleanNullFractional", ["DataType", "att1", N], {"DataTypeHistogram": [1, 1, 0, 2, 0]}, S + ":405-421", []),
    ("dataWithNullColumns", ["DataType", "stringCol", N], {"DataTypeHistogram": [8, 0, 0, 0, 0]}, "analyzers/NullHandlingTests.scala:69-70", []),
    # incremental (analyzers/IncrementalAnalyzerTest.scala:49-99)
    ("incrementalInitial", ["Size", N], 3.0, "analyzers/IncrementalAnalyzerTest.scala:58", []),
    ("incrementalInitial", ["Completeness", "att1", N], 0.6666666666666666, "analyzers/IncrementalAnalyzerTest.scala:96", []),
    ("incrementalInitial", ["Compliance", "att1", "att1 = 'b'", N], 0.3333333333333333, "analyzers/IncrementalAnalyzerTest.scala:77", []),
    # PatternMatch: "regex_fallback" = outside the GPU regex subset / a non-string column (Spark path)
    ("patternDoubles", ["PatternMatch", "some", r"\d\.\d", N], 0.75, S + ":628-631", ["regex_fallback"]),
    ("patternIntegers", ["PatternMatch", "some", r"\d", N], 0.5, S + ":634-637", []),
    ("patternEmails", ["PatternMatch", "some", EMAIL, N], 0.5, S + ":640-643", []),
    ("patternCreditCards", ["PatternMatch", "some", CREDITCARD, N], 10.0 / 13.0, S + ":646-671", ["regex_fallback"]),
    ("patternUrls", ["PatternMatch", "some", URL, N], 10.0 / 13.0, S + ":673-699", []),
    ("patternSsns", ["PatternMatch", "some", SSN, N], 2.0 / 8.0, S + ":701-718", ["regex_fallback"]),
    ("checkUrls", ["PatternMatch", "some", URL, N], 0.5, "checks/CheckTest.scala:381-389 (hasPattern default assertion fails)", []),
    ("checkEmails", ["PatternMatch", "some", EMAIL, N], 1.0, "checks/CheckTest.scala:352-360 (hasPattern default assertion holds)", []),
    # grouping analyzers (AnalyzerTests.scala:79-146, AnalysisTest.scala:30-93, NullHandlingTests.scala:112-115)
    ("dfMissing", ["Uniqueness", ["att1"]], 0.0, S + ":84-85", []),
    ("dfMissing", ["Uniqueness", ["att2"]], 0.0, S + ":86-87", []),
    ("dfFull", ["Uniqueness", ["att1"]], 0.25, S + ":90-91", []),
    ("dfFull", ["Uniqueness", ["att2"]], 0.25, S + ":92-93", []),
    ("dfWithUniqueColumns", ["Uniqueness", ["unique"]], 1.0, S + ":99-100", []),
    ("dfWithUniqueColumns", ["Uniqueness", ["uniqueWithNulls"]], 5 / 6.0, S + ":101-102", []),
    ("dfWithUniqueColumns", ["Uniqueness", ["unique", "nonUnique"]], 1.0, S + ":103-104", []),
    ("dfWithUniqueColumns", ["Uniqueness", ["unique", "nonUniqueWithNulls"]], 3 / 6.0, S + ":105-107", []),
    ("dfWithUniqueColumns", ["Uniqueness", ["nonUnique", "onlyUniqueWithOtherNonUnique"]], 1.0, S + ":108-110", []),
    ("dfFull", ["Entropy", "att1"], -(0.75 * math.log(0.75) + 0.25 * math.log(0.25)), S + ":138-140", []),
    ("dfFull", ["Entropy", "att2"], -(0.75 * math.log(0.75) + 0.25 * math.log(0.25)), S + ":141-143", []),
    ("dfFull", ["Distinctness", ["item"]], 1.0, "analyzers/AnalysisTest.scala:38,49", []),
    ("dfFull", ["Uniqueness", ["att1", "att2"]], 0.25, "analyzers/AnalysisTest.scala:40,51", []),
    ("dfWithNumericValues", ["CountDistinct", ["att1"]], 6.0, "analyzers/AnalysisTest.scala:80,93", []),
    ("dfWithUniqueColumns", ["CountDistinct", ["uniqueWithNulls"]], 5.0, S + ":526-529", []),
    ("dataWithNullColumns", ["CountDistinct", ["stringCol"]], 0.0, "analyzers/NullHandlingTests.scala:112", []),
    ("dataWithNullColumns", ["Entropy", "stringCol"], "EmptyState", "analyzers/NullHandlingTests.scala:115", []),
    ("dfFull", ["MutualInformation", ["att1", "att2"]], -(0.75 * math.log(0.75) + 0.25 * math.log(0.25)), S + ":148-152", []),
    ("dfWithConditionallyUninformativeColumns", ["MutualInformation", ["att1", "att2"]], 0.0, S + ":153-156", []),
    ("dfFull", ["MutualInformation", ["att1", "att1"]], -(0.75 * math.log(0.75) + 0.25 * math.log(0.25)), S + ":157-167 (equals Entropy(att1))", []),
    ("dataWithNullColumns", ["MutualInformation", ["numericCol", "numericCol2"]], "EmptyState", "analyzers/NullHandlingTests.scala:116", []),
    ("dataWithNullColumns", ["MutualInformation", ["numericCol", "numericCol3"]], "EmptyState", "analyzers/NullHandlingTests.scala:117", []),
    # column types beyond Int / Long / Double (round 6): checks/CheckTest.scala:478-489 via :765-785 -- the
    # default assertion of isNonNegative / isPositive is `_ == 1.0` (Check.scala:670-688), and the checks succeed
    *[(f"numericRowNull_{t}", ["Compliance", "some is non-negative", "COALESCE(some, 0.0) >= 0", N], 1.0,
       "checks/CheckTest.scala:478-482,765-785 (isNonNegative succeeds; predicate form Check.scala:676)", [])
      for t in ("i8", "i16", "i32", "i64", "f32", "f64")],
    *[(f"numericRowNull_{t}", ["Compliance", "some is positive", "COALESCE(some, 1.0) > 0", N], 1.0,
       "checks/CheckTest.scala:484-488,765-785 (isPositive succeeds; predicate form Check.scala:687)", [])
      for t in ("i8", "i16", "i32", "i64", "f32", "f64")],
    ("dfWithNumericValuesAsFloat", ["DataType", "att1_float", N], {"DataTypeHistogram": [0, 6, 0, 0, 0]}, S + ":322-328", []),
    ("dfBooleanColumn", ["Completeness", "attribute", N], 5.0 / 6.0,
     "profiles/ColumnProfilerTest.scala:177-190 fixture; expected value computed by hand (5 of 6 non-null)", []),
    ("dfBooleanColumn", ["DataType", "attribute", N], {"DataTypeHistogram": [1, 0, 0, 5, 0]},
     "profiles/ColumnProfilerTest.scala:177-190 fixture; StatefulDataType.scala:62-67 on \"true\" / \"false\" (by hand)", []),
    ("dfBooleanColumn", ["ApproxCountDistinct", "attribute", N], 2.0,
     "profiles/ColumnProfilerTest.scala:177-190 fixture (two distinct values); expected value computed by hand", []),
    ("dfDecimalSystemDefault", ["Minimum", "num", N], 99.0, S + ":489-505 (Minimum on decimal columns)", []),
    # DataType constraints (constraints/ConstraintsTest.scala:126-146): Fractional ratio 1.0 of a DoubleType column;
    # Fractional 0.5 and Numeric (fractional + integral) 1.0 of a StringType column of "1" and "2.0"
    ("dfDoubleColumn", ["DataType", "column", N], {"DataTypeHistogram": [0, 2, 0, 0, 0]},
     "constraints/ConstraintsTest.scala:126-130", []),
    ("dfStringNumericColumn", ["DataType", "column", N], {"DataTypeHistogram": [0, 1, 1, 0, 0]},
     "constraints/ConstraintsTest.scala:132-136,143-146", []),
    # partition merge (analyzers/StateAggregationIntegrationTest.scala:56-104)
    ("stateAggregation", ["Completeness", "origin", N], 0.625, "analyzers/StateAggregationIntegrationTest.scala:77", []),
]

out = {
    "doc": __doc__,
    "datasets": datasets,
    "cases": [
        {"dataset": d, "analyzer": a, "expected": e, "source": s, "needs": nd}
        for (d, a, e, s, nd) in cases
    ],
}

if __name__ == "__main__":
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(dst, len(cases))
