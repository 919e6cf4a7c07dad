"""Default flow document and metrics dashboard template (the role of the reference's
Services/DataX.Config/CommonData.Templates/defaultFlowConfig.json): every flow gets the built-in event-rate metric
``DATAX-<flow>:Input_DataXProcessedInput_Events_Count`` charted as events/second, total and average."""
from __future__ import annotations

from typing import Any, Dict


def default_flow(name: str) -> Dict[str, Any]:
    key = f"DATAX-{name}:Input_DataXProcessedInput_Events_Count"
    return {
        "name": name,
        "displayName": name,
        "commonProcessor": {"jobCommonTokens": {"jobName": name, "engineJobName": f"dxa-{name}"},
                            "jobs": [{"partitionJobNumber": "1"}]},
        "metrics": {
            "sources": [{"name": "events", "input": {"type": "MetricApi", "metricKeys": [key]},
                         "output": {"type": "SumWithTimeChart",
                                    "data": {"sum": True, "timechart": True, "average": True, "speed": True},
                                    "dynamicOffsetInMs": 300000}}],
            "widgets": [
                {"name": "eventsChart", "displayName": "Events/Second", "data": "events_timechart",
                 "position": "TimeCharts", "type": "StackAreaChart"},
                {"name": "totalEvents", "displayName": "Events Ingested Today", "data": "events_sum",
                 "formatter": "longint", "position": "FirstRow", "type": "SimpleBox"},
                {"name": "averageEvents", "displayName": "Avg. Events/Minute", "data": "events_average",
                 "formatter": "longint", "position": "FirstRow", "type": "SimpleBox"}],
            "initParameters": {"widgetSets": ["direct"], "jobNames": {"type": "getCPSparkJobNames"}},
        },
    }
