// Flow designer model: option lists and defaults for each tab (the role of datax-pipeline flowModels.js). The
// designer edits the flow in the reference's UI shape (newFlow below); designer/flow/toconfig turns it into the
// product config that flow/save stores and the config generator (dxa/flow/configgen.py) consumes.

const opt = (key, name) => ({ key, name });

export const inputModes = [opt('streaming', 'Streaming'), opt('batching', 'Batching')];

export const inputTypes = [
    opt('events', 'Event Hub'),
    opt('iothub', 'IoT Hub'),
    opt('kafka', 'Kafka'),
    opt('kafkaeventhub', 'Kafka (Event Hub)'),
    opt('local', 'Local generator'),
    opt('socket', 'Socket'),
    opt('file', 'Files')
];
export const inputTypesBatching = [opt('blob', 'Azure Blob / files')];

export const watermarkUnits = [opt('second', 'Seconds'), opt('minute', 'Minutes'), opt('hour', 'Hours')];
export const formatTypes = [opt('json', 'JSON')];
export const inputCompressionTypes = [opt('none', 'None'), opt('gzip', 'GZip')];
export const referenceDataTypes = [opt('csv', 'CSV/TSV File')];
export const csvDelimiters = [opt(',', 'Comma'), opt('\t', 'Tab')];

export const functionTypes = [
    opt('hipUDF', 'HIP UDF (GPU)'),
    opt('hipUDAF', 'HIP UDAF (GPU)'),
    opt('jarUDF', 'UDF (class)'),
    opt('jarUDAF', 'UDAF (class)'),
    opt('azureFunction', 'Azure Function')
];
export const functionMethodTypes = [opt('get', 'Get'), opt('post', 'Post')];
export const udfValueTypes = ['double', 'long', 'int', 'boolean', 'string'].map(t => opt(t, t));

export const sinkerTypes = [
    opt('blob', 'Azure Blob'),
    opt('cosmosdb', 'Cosmos DB'),
    opt('eventhub', 'Event Hub'),
    opt('sql', 'SQL Server / Azure SQL'),
    opt('local', 'Local files'),
    opt('httppost', 'HTTP POST'),
    opt('console', 'Console')
];
export const sinkerCompressionTypes = [opt('none', 'None'), opt('gzip', 'GZip')];
export const sinkerFormatTypes = [opt('json', 'JSON')];
export const sqlWriteModes = [opt('append', 'Append'), opt('overwrite', 'Overwrite'), opt('ignore', 'Ignore'),
    opt('errorifexists', 'Error if exists')];

export const batchTypes = [opt('recurring', 'Recurring'), opt('oneTime', 'One Time')];
export const batchIntervalTypes = [opt('day', 'Day'), opt('hour', 'Hour'), opt('min', 'Min')];

export const ruleSubTypes = [opt('SimpleRule', 'Simple rule'), opt('AggregateRule', 'Aggregate rule')];
export const aggregateTypes = ['AVG', 'COUNT', 'DCOUNT', 'MAX', 'MIN', 'SUM'].map(a => opt(a, a));
// a condition of an aggregate rule either aggregates its field or ('none') groups by it
export const conditionAggregateTypes = [opt('none', '(group by)')].concat(aggregateTypes);
export const conjunctionTypes = [opt('and', 'AND'), opt('or', 'OR')];
export const severityTypes = [opt('Critical', 'Critical'), opt('Medium', 'Medium'), opt('Low', 'Low')];
export const numberOperators = [
    opt('equal', '='), opt('notEqual', '!='), opt('greater', '>'), opt('lessThan', '<'),
    opt('greaterThanOrEqual', '>='), opt('lessThanOrEqual', '<=')
];
export const stringOperators = [
    opt('stringEqual', 'equals'), opt('stringNotEqual', 'not equals'), opt('contains', 'contains'),
    opt('notContains', 'does not contain'), opt('startsWith', 'starts with'), opt('endsWith', 'ends with')
];

export const metricSinkerName = 'Metrics';
export const defaultSchemaTableName = 'DataXProcessedInput';

export const defaultNormalizationSnippet = 'SystemProperties AS _SystemProperties\nProperties AS _Properties\nRaw.*';
export const defaultBatchNormalizationSnippet = 'Raw.*';

export const defaultSchema = JSON.stringify(
    {
        type: 'struct',
        fields: [
            { name: 'deviceId', type: 'long', nullable: true, metadata: {} },
            { name: 'temperature', type: 'double', nullable: true, metadata: {} },
            { name: 'eventTime', type: 'string', nullable: true, metadata: {} }
        ]
    },
    null,
    2
);

export const defaultSchemaLocal = JSON.stringify(
    {
        type: 'struct',
        fields: [
            { name: 'temperature', type: 'double', nullable: false, metadata: { minValue: 5.1, maxValue: 100.1 } },
            { name: 'eventTime', type: 'long', nullable: false, metadata: { useCurrentTimeMillis: true } }
        ]
    },
    null,
    2
);

export const defaultQuery = '--DataXQuery--\nT1 = SELECT * FROM DataXProcessedInput;\n\nOUTPUT T1 TO Metrics;';

export function defaultInput(onebox) {
    return {
        type: onebox ? 'local' : 'events',
        mode: 'streaming',
        properties: {
            inputEventhubName: '',
            inputEventhubConnection: '',
            windowDuration: '30',
            timestampColumn: '',
            watermarkValue: '0',
            watermarkUnit: 'second',
            maxRate: onebox ? '100' : '1000',
            inputSchemaFile: onebox ? defaultSchemaLocal : defaultSchema,
            normalizationSnippet: defaultNormalizationSnippet
        }
    };
}

export function defaultDisplayName() {
    return 'test' + (Math.floor(Math.random() * 90000) + 10000);
}

// The designer model of a flow (designer.config_to_flow / flowHelpers.convertConfigToFlow): flow/get's config is
// converted to it on load, and designer/flow/toconfig converts it back before flow/save.
export function newFlow(onebox, owner) {
    return {
        name: '',
        flowId: '',
        displayName: defaultDisplayName(),
        owner: owner || '',
        databricksToken: '',
        input: defaultInput(onebox),
        batchInputs: [defaultBatchInput()],
        batchList: [],
        referenceData: [],
        functions: [],
        query: defaultQuery,
        scale: { jobNumGpus: '1' },
        outputs: [metricSinker()],
        outputTemplates: [],
        rules: []
    };
}

// fill the parts an older or hand-written document may lack, so every tab can render it
export function normalizeFlow(flow) {
    const base = newFlow(false, flow.owner);
    for (const k of Object.keys(base)) if (flow[k] === undefined || flow[k] === null) flow[k] = base[k];
    flow.input.properties = Object.assign(defaultInput(false).properties, flow.input.properties || {});
    flow.input.type = flow.input.type || 'events';
    flow.input.mode = flow.input.mode || 'streaming';
    if (!flow.batchInputs.length) flow.batchInputs = [defaultBatchInput()];
    flow.scale = Object.assign({ jobNumGpus: '1' }, flow.scale || {});
    for (const r of flow.rules) {
        r.properties.aggs = r.properties.aggs || [];
        r.properties.pivots = r.properties.pivots || [];
        r.properties.alertSinks = r.properties.alertSinks || [];
        r.properties.conditions = r.properties.conditions || defaultGroup();
    }
    return flow;
}

export function metricSinker() {
    return { id: metricSinkerName, type: 'metric', properties: {} };
}

export function defaultBatchInput() {
    return { type: 'blob', properties: { connection: '', path: '', formatType: 'json', compressionType: 'none' } };
}

export function defaultReferenceData() {
    return { id: '', type: 'csv', properties: { path: '', delimiter: ',', header: true } };
}

export function defaultFunction(type) {
    if (type === 'azureFunction') {
        return { id: '', type, properties: { serviceEndpoint: '', api: '', code: '', methodType: 'get', params: [] } };
    }
    if (type === 'hipUDF') {
        return {
            id: '',
            type,
            properties: {
                source: '__device__ double myudf(double x) { return x * 2.0; }',
                entry: '',
                returnType: 'double',
                argTypes: ['double'],
                nullSafe: false
            }
        };
    }
    if (type === 'hipUDAF') {
        return {
            id: '',
            type,
            properties: {
                source: 'struct State { double s; };\n__device__ void init(State& st) { st.s = 0; }\n' +
                    '__device__ void update(State& st, double x) { st.s += x; }\n' +
                    '__device__ void merge(State& a, const State& b) { a.s += b.s; }\n' +
                    '__device__ double finish(const State& st) { return st.s; }',
                prefix: '',
                returnType: 'double',
                argTypes: ['double'],
                nullSafe: false
            }
        };
    }
    return { id: '', type, properties: { path: '', class: '', libs: [] } };
}

export function defaultSinker(type) {
    switch (type) {
        case 'cosmosdb':
            return { id: '', type, properties: { connectionString: '', db: '', collection: '' } };
        case 'eventhub':
            return { id: '', type, properties: { connectionString: '', format: 'json', compressionType: 'gzip' } };
        case 'blob':
            return {
                id: '',
                type,
                properties: { connectionString: '', containerName: '', blobPrefix: '', blobPartitionFormat: 'yyyy/MM/dd/HH',
                    format: 'json', compressionType: 'gzip' }
            };
        case 'local':
            return {
                id: '',
                type,
                properties: { folder: '', blobPrefix: '', blobPartitionFormat: 'yyyy/MM/dd/HH', format: 'json', compressionType: 'none' }
            };
        case 'sql':
            return { id: '', type, properties: { connectionString: '', databaseName: '', tableName: '', writeMode: 'append', useBulkInsert: false } };
        case 'httppost':
            return { id: '', type, properties: { endpoint: '', filter: '' } };
        case 'console':
            return { id: '', type, properties: { maxRows: 20 } };
        default:
            return { id: '', type, properties: {} };
    }
}

export function defaultBatch(type) {
    return {
        id: '',
        type,
        disabled: false,
        properties: {
            interval: '1',
            intervalType: 'day',
            delay: '0',
            delayType: 'day',
            window: '1',
            windowType: 'day',
            startTime: type === 'oneTime' ? '' : new Date().toISOString().slice(0, 19) + 'Z',
            endTime: '',
            lastProcessedTime: ''
        }
    };
}

export function defaultCondition() {
    return { type: 'condition', conjunction: 'and', aggregate: 'none', field: '', operator: 'equal', value: '' };
}

export function defaultGroup() {
    return { type: 'group', conjunction: 'and', conditions: [defaultCondition()] };
}

export function defaultRule() {
    return {
        id: '',
        type: 'tag',
        properties: {
            productId: '',
            ruleType: 'SimpleRule',
            ruleId: '',
            ruleDescription: '',
            condition: '',
            tagName: 'Tag',
            tag: '',
            aggs: [],
            pivots: [],
            isAlert: false,
            severity: 'Critical',
            alertSinks: [],
            outputTemplate: '',
            schemaTableName: defaultSchemaTableName,
            conditions: defaultGroup()
        }
    };
}
