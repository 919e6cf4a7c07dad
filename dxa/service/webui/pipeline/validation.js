// Per-tab completeness checks of the flow designer (the role of datax-pipeline flowSelectors.js validate*). A tab
// whose settings are incomplete gets a marker, and Deploy stays disabled until every tab is complete.

export const isValidNumberAboveZero = v => v !== undefined && v !== null && String(v).trim() !== '' && isFinite(v) && Number(v) > 0;
export const isValidNumberAboveOrEqualZero = v =>
    v !== undefined && v !== null && String(v).trim() !== '' && isFinite(v) && Number(v) >= 0;
export const isNumberAndStringOnly = v => typeof v === 'string' && /^[A-Za-z0-9]+$/.test(v);
const nonEmpty = v => typeof v === 'string' ? v.trim() !== '' : v !== undefined && v !== null && v !== '';

export function isValidJson(text) {
    try {
        JSON.parse(text);
        return true;
    } catch (e) {
        return false;
    }
}

const NUMBER_OPS = new Set(['equal', 'notEqual', 'greater', 'lessThan', 'greaterThanOrEqual', 'lessThanOrEqual']);

// flowHelpers isConditionsValid: message of the first violation, or null
export function conditionsError(group, ruleType) {
    function cond(c) {
        if (ruleType === 'AggregateRule' && c.aggregate && c.aggregate !== 'none' && !NUMBER_OPS.has(c.operator))
            return 'Text operators cannot be used with Aggregate conditions';
        if (!nonEmpty(c.field)) return 'All conditions need to have column name specified';
        if (!nonEmpty(c.value)) return 'All conditions need to have a value specified';
        if (NUMBER_OPS.has(c.operator) && !(isFinite(c.value) && String(c.value).trim() !== ''))
            return 'Value field must be a number when a numeric operator is used';
        return null;
    }
    function grp(g) {
        if (!g.conditions || !g.conditions.length) return 'All groups need to have at least 1 condition';
        for (const c of g.conditions) {
            const e = c.type === 'group' ? grp(c) : cond(c);
            if (e) return e;
        }
        return null;
    }
    return group ? grp(group) : 'rule has no conditions';
}

export function validateInfo(flow) {
    return nonEmpty(flow.displayName);
}

export function validateInput(flow) {
    const input = flow.input;
    if (!input || !input.properties) return false;
    if (input.mode === 'batching') return (flow.batchInputs || []).length > 0 && flow.batchInputs.every(isBatchInputComplete);
    if (input.mode !== 'streaming') return false;
    const p = input.properties;
    const common = [
        isValidNumberAboveZero(p.windowDuration),
        isValidNumberAboveOrEqualZero(p.watermarkValue),
        isValidNumberAboveZero(p.maxRate),
        isValidJson(p.inputSchemaFile)
    ];
    switch (input.type) {
        case 'events':
            return common.concat([nonEmpty(p.inputEventhubConnection)]).every(Boolean);
        case 'iothub':
        case 'kafka':
        case 'kafkaeventhub':
            return common.concat([nonEmpty(p.inputEventhubName), nonEmpty(p.inputEventhubConnection)]).every(Boolean);
        case 'socket':
        case 'file':
            return common.concat([nonEmpty(p.inputEventhubConnection)]).every(Boolean);
        case 'local':
            return common.every(Boolean);
        default:
            return false;
    }
}

export function isBatchInputComplete(b) {
    if (!b || !b.properties || b.type !== 'blob') return false;
    const p = b.properties;
    return [nonEmpty(p.path), nonEmpty(p.formatType), nonEmpty(p.compressionType)].every(Boolean);
}

export function isReferenceDataComplete(r) {
    if (!r || !r.properties || !isNumberAndStringOnly(r.id)) return false;
    return r.type === 'csv' && nonEmpty(r.properties.path);
}

export function validateReferenceData(flow) {
    return (flow.referenceData || []).every(isReferenceDataComplete);
}

export function isFunctionComplete(f) {
    if (!f || !f.properties || !isNumberAndStringOnly(f.id)) return false;
    const p = f.properties;
    switch (f.type) {
        case 'jarUDF':
        case 'jarUDAF':
            return nonEmpty(p.path) && nonEmpty(p.class) && (p.libs || []).every(nonEmpty);
        case 'hipUDF':
        case 'hipUDAF':
            return nonEmpty(p.source) && nonEmpty(p.returnType) && (p.argTypes || []).every(nonEmpty);
        case 'azureFunction':
            return nonEmpty(p.serviceEndpoint) && nonEmpty(p.api) && nonEmpty(p.methodType) && (p.params || []).every(nonEmpty);
        default:
            return false;
    }
}

export function validateFunctions(flow) {
    return (flow.functions || []).every(isFunctionComplete);
}

export function isSinkerComplete(o) {
    if (!o || !o.properties || !isNumberAndStringOnly(o.id)) return false;
    const p = o.properties;
    switch (o.type) {
        case 'cosmosdb':
            return nonEmpty(p.connectionString) && isNumberAndStringOnly(p.db || '') && isNumberAndStringOnly(p.collection || '');
        case 'eventhub':
            return nonEmpty(p.connectionString);
        case 'blob':
            return nonEmpty(p.connectionString) && isNumberAndStringOnly(p.containerName || '') && nonEmpty(p.blobPrefix) &&
                nonEmpty(p.blobPartitionFormat);
        case 'local':
            return nonEmpty(p.folder) || nonEmpty(p.connectionString);
        case 'sql':
            return nonEmpty(p.connectionString) && nonEmpty(p.tableName);
        case 'httppost':
            return nonEmpty(p.endpoint);
        case 'metric':
        case 'console':
            return true;
        default:
            return false;
    }
}

export function validateOutputs(flow) {
    return (flow.outputs || []).length > 0 && flow.outputs.every(isSinkerComplete);
}

export function isOutputTemplateComplete(t) {
    return !!t && nonEmpty(t.id) && nonEmpty(t.template);
}

export function isRuleComplete(r) {
    if (!r || !r.properties || !nonEmpty(r.id) || r.type !== 'tag') return false;
    const p = r.properties;
    if (!nonEmpty(p.ruleDescription)) return false;
    if (p.isAlert && !(p.alertSinks || []).length) return false;
    if (conditionsError(p.conditions, p.ruleType)) return false;
    if (p.ruleType === 'AggregateRule') {
        if (!(p.aggs || []).every(a => nonEmpty(a.column))) return false;
        if (!(p.pivots || []).every(nonEmpty)) return false;
    }
    return true;
}

export function validateRules(flow) {
    return (flow.rules || []).every(isRuleComplete) && (flow.outputTemplates || []).every(isOutputTemplateComplete);
}

export function validateScale(flow) {
    const n = flow.scale && flow.scale.jobNumGpus;
    return isValidNumberAboveZero(n) && Number.isInteger(Number(n));
}

export function isBatchComplete(b) {
    if (!b || !b.properties || !isNumberAndStringOnly(b.id)) return false;
    const p = b.properties;
    const base = [nonEmpty(p.interval), nonEmpty(p.intervalType), nonEmpty(p.delayType), nonEmpty(p.window),
        nonEmpty(p.windowType), nonEmpty(p.startTime), isValidNumberAboveZero(p.interval), isValidNumberAboveZero(p.window)];
    if (b.type === 'recurring') return base.concat([isValidNumberAboveOrEqualZero(p.delay)]).every(Boolean);
    if (b.type === 'oneTime') return base.concat([Number(p.delay) === 0, nonEmpty(p.endTime)]).every(Boolean);
    return false;
}

export function validateSchedule(flow) {
    return (flow.input && flow.input.mode === 'streaming') || ((flow.batchList || []).length > 0 && flow.batchList.every(isBatchComplete));
}

export function validateQuery(flow) {
    return nonEmpty(flow.query);
}

export const TAB_VALIDATORS = {
    info: validateInfo,
    input: validateInput,
    referenceData: validateReferenceData,
    functions: validateFunctions,
    query: validateQuery,
    rules: validateRules,
    outputs: validateOutputs,
    scale: validateScale,
    schedule: validateSchedule
};

export function validateFlow(flow) {
    return Object.keys(TAB_VALIDATORS).every(k => TAB_VALIDATORS[k](flow));
}
